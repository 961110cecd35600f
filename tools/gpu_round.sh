# Round measurement: GPU tests, the default bench (20 GB, with cpu_baseline), a rocprofv3
# kernel-trace/stats pass, and FETCH_SIZE (PMC) passes of the same workload: normal and with
# K1 in load-only mode (TSG_DIAG_SCAN=2: reads exactly the arena -> FETCH_SIZE calibration).
# Usage: gpurun -- 'TAG=r01v5 bash tools/gpu_round.sh'
set -o pipefail
TAG=${TAG:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_bench_$TAG.json 2> $R/gpurun_out/prof_$TAG.err
rc=$?; cd $R; tail -2 gpurun_out/prof_$TAG.err; [ $rc -eq 0 ] || exit $rc
cat gpurun_out/prof_bench_$TAG.json
find gpurun_out/prof_$TAG -name '*kernel_stats.csv' -exec cat {} \;
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_$TAG -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_bench_$TAG.json 2> $R/gpurun_out/pmc_$TAG.err
rc=$?; cd $R; tail -2 gpurun_out/pmc_$TAG.err; [ $rc -eq 0 ] || exit $rc
cd /tmp
TSG_DIAG_SCAN=2 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_${TAG}_diag2 -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_bench_${TAG}_diag2.json 2> $R/gpurun_out/pmc_${TAG}_diag2.err
rc=$?; cd $R; tail -2 gpurun_out/pmc_${TAG}_diag2.err; exit $rc
