# C2 pipeline depth 3 vs 4, interleaved, 50 timed steps each
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03s}
for dp in 3 4 3 4 3 4; do
  timeout -k 10 300 python bench.py --depth $dp --no-cpu-baseline --ingest-steps 0 > gpurun_out/bench_${T}_d$dp.json 2> gpurun_out/bench_${T}_d$dp.err
  rc=$?; python -c "import json;d=json.load(open('gpurun_out/bench_${T}_d$dp.json'));b=d['breakdown_ms'];print('depth=$dp',d['value'],d['ms_per_step'],b['ms_gpu_total'],b['ms_scan_kernel'],d['host_cpu']['process_cpu_ms_per_step'],d['host_cpu']['cpus_used'])"; [ $rc -eq 0 ] || exit $rc
done
