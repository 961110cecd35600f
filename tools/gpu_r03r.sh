# C2 default bench at 50 timed steps; pipeline depth A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03r}
timeout -k 10 600 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; python tools/bench_brief.py gpurun_out/bench_$T.json; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/bench_$T.json'));print(d['value'],d['steps'],d['ms_per_step'],d['host_cpu']['process_cpu_ms_per_step'],d['host_cpu']['cpus_used'],(d.get('parity') or {}).get('mismatches'),(d.get('cpu_baseline') or {}).get('value'),(d.get('ingest') or {}).get('value'),d['roofline']['frac'])"
for dp in 2 4 3; do
  timeout -k 10 300 python bench.py --depth $dp --no-cpu-baseline --ingest-steps 0 > gpurun_out/bench_${T}_d$dp.json 2> gpurun_out/bench_${T}_d$dp.err
  rc=$?; echo "depth=$dp"; python -c "import json;d=json.load(open('gpurun_out/bench_${T}_d$dp.json'));print(d['value'],d['ms_per_step'],d['breakdown_ms']['ms_gpu_total'],d['host_cpu']['process_cpu_ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
done
