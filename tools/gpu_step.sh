# One iteration: -m gpu suite, default bench (10 steps), then a 1-scan 20 GB run that dumps the GPU
# candidates (host-tail profiling on the CPU: tools/host_tail_bench.py) with the tail phase timers on.
# Usage: gpurun -- 'TAG=r02x bash tools/gpu_step.sh'
set -o pipefail
TAG=${TAG:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; python tools/bench_brief.py gpurun_out/bench_$TAG.json; tail -2 gpurun_out/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc
if [ -n "${DUMP:-}" ]; then
  TSG_TAIL_DEBUG=1 TSG_DUMP_CANDS=$GRAFT_REPO_ROOT/gpurun_out/cands_20g.bin timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/dump_$TAG.json 2> gpurun_out/dump_$TAG.err
  rc=$?; tail -6 gpurun_out/dump_$TAG.err; exit $rc
fi
