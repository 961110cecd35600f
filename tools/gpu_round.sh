# parity tests, then the 20 GB bench, then a rocprofv3 kernel-trace of a 4 GB bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_parity.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 3 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
if [ -n "${PROFILE:-}" ]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --gb 4 --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err
  rc=$?; cd $GRAFT_REPO_ROOT; tail -3 gpurun_out/prof.err; find gpurun_out/prof -name '*stats*' | head; exit $rc
fi
