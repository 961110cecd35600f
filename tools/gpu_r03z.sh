# Final tree workloads (one line each) and the default bench with its CPU baseline and ingest leg
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03z}
for wl in c3 c3f c4 c1fs c5; do
  timeout -k 10 500 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_$wl.json 2> gpurun_out/wl_${T}_$wl.err
  rc=$?; echo "== $wl"; python tools/bench_brief.py gpurun_out/wl_${T}_$wl.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; python tools/bench_brief.py gpurun_out/bench_$T.json; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/bench_$T.json'));print(d['value'],d['steps'],d['ms_per_step'],d['host_cpu']['process_cpu_ms_per_step'],(d.get('parity') or {}).get('mismatches'),(d.get('parity') or {}).get('files'),(d.get('cpu_baseline') or {}).get('value'),(d.get('ingest') or {}).get('value'),d['roofline']['frac'])"
