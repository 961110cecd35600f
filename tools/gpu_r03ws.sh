# Default bench (now with a 10-s time-based warm-up) twice on one box, as the driver runs it
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03ws}
for i in 1 2; do
  timeout -k 10 600 python bench.py > gpurun_out/bench_${T}_$i.json 2> gpurun_out/bench_${T}_$i.err
  rc=$?; python tools/bench_brief.py gpurun_out/bench_${T}_$i.json; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/bench_${T}_$i.json'));print(d['value'],d['warmup'],d['steps'],d['ms_per_step'],(d.get('parity') or {}).get('mismatches'),(d.get('cpu_baseline') or {}).get('value'),(d.get('ingest') or {}).get('value'))"
done
