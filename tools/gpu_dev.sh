# Development loop: GPU tests, default bench, per-item diagnostics at C2, rocprof kernel stats.
# Usage: gpurun -- 'TAG=r02b bash tools/gpu_dev.sh'
set -o pipefail
TAG=${TAG:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/items_$TAG.txt
TSG_DIAG_ITEMS=$R/gpurun_out/items_$TAG.txt timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bench_diag_$TAG.json 2> gpurun_out/bench_diag_$TAG.err
rc=$?; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_bench_$TAG.json 2> $R/gpurun_out/prof_$TAG.err
rc=$?; cd $R; tail -2 gpurun_out/prof_$TAG.err; [ $rc -eq 0 ] || exit $rc
find gpurun_out/prof_$TAG -name '*kernel_stats.csv' -exec cat {} \;
