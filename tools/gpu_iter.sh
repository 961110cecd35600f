# Iteration loop: GPU tests, the 20 GB bench (no CPU baseline), K1 diag modes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
if [ -n "${DIAG:-}" ]; then
  for m in 1 2; do
    TSG_DIAG_SCAN=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/k1_diag$m.json 2> gpurun_out/k1_diag$m.err || exit $?
    echo "diag $m"; cat gpurun_out/k1_diag$m.json
  done
fi
