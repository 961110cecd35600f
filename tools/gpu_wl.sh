# Workload check: GPU tests, then c2 / c3 / c4 benches (no CPU baseline unless CPU=1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
CB=--no-cpu-baseline; [ -n "${CPU:-}" ] && CB=
for wl in ${WLS:-c2 c3 c4}; do
  timeout -k 10 600 python bench.py --workload $wl --steps 3 --warmup 1 $CB ${BENCH_ARGS:-} > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err
  rc=$?; echo "== $wl"; cat gpurun_out/bench_$wl.json; tail -3 gpurun_out/bench_$wl.err; [ $rc -eq 0 ] || exit $rc
done
