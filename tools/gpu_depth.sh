# Pipeline-depth sweep of the default bench (no CPU baseline) + the multi-rank GPU test.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_multirank.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_multirank.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_multirank.log; [ $rc -eq 0 ] || exit $rc
for d in ${DEPTHS:-2 3 4}; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --depth $d --no-cpu-baseline > gpurun_out/bench_depth$d.json 2> gpurun_out/bench_depth$d.err
  rc=$?; echo "== depth $d"; cut -c1-420 gpurun_out/bench_depth$d.json; tail -2 gpurun_out/bench_depth$d.err; [ $rc -eq 0 ] || exit $rc
done
