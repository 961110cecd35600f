# Pipeline-depth sweep of the default bench (no CPU baseline, no ingest leg):
# value, ms/step and the per-scan latency split for each depth.
#   gpurun -- 'DEPTHS="2 3 4" bash tools/gpu_depth.sh'   (MULTIRANK=1 adds the multi-rank GPU test)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${MULTIRANK:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_multirank.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_multirank.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_multirank.log; [ $rc -eq 0 ] || exit $rc
fi
echo "depth value ms_per_step gpu_total host_gpu_phase host_exact host_total"
for d in ${DEPTHS:-2 3 4}; do
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --ingest-steps 0 --depth $d > gpurun_out/depth_$d.json 2> gpurun_out/depth_$d.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/depth_$d.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/depth_$d.json'));b=d['breakdown_ms'];print($d, d['value'], d['ms_per_step'], b['ms_gpu_total'], b['ms_host_gpu_phase'], b['ms_host_exact'], b['ms_host_total'])"
done
