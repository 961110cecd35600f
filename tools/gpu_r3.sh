# Round-3 iteration on the GPU box: -m gpu tests, the default bench, optional
# workloads and a rocprof kernel-stats pass.  Every GPU step has its own time
# limit; the script stops at the first failure.
#   gpurun -- 'TAG=r03a WLS="c3" PROF=1 bash tools/gpu_r3.sh'
set -o pipefail
TAG=${TAG:-r03}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; python tools/bench_brief.py gpurun_out/bench_$TAG.json 2>/dev/null || cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc
fi
for wl in ${WLS:-}; do
  timeout -k 10 600 python bench.py --workload $wl --steps ${WL_STEPS:-5} --warmup 1 --no-cpu-baseline > gpurun_out/wl_${TAG}_$wl.json 2> gpurun_out/wl_${TAG}_$wl.err
  rc=$?; python tools/bench_brief.py gpurun_out/wl_${TAG}_$wl.json 2>/dev/null || cat gpurun_out/wl_${TAG}_$wl.json; tail -3 gpurun_out/wl_${TAG}_$wl.err; [ $rc -eq 0 ] || exit $rc
done
if [ -n "${PROF:-}" ]; then
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --ingest-steps 0 > $R/gpurun_out/prof_bench_$TAG.json 2> $R/gpurun_out/prof_$TAG.err
  rc=$?; cd $R; tail -2 gpurun_out/prof_$TAG.err; [ $rc -eq 0 ] || exit $rc
  find gpurun_out/prof_$TAG -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-8 | head -20
fi
