set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_r03b.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r03b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r03b.json 2> gpurun_out/bench_r03b.err
rc=$?; python tools/bench_brief.py gpurun_out/bench_r03b.json; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r03b_c4 -o run --output-format csv -- python3 $R/bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_bench_r03b_c4.json 2> $R/gpurun_out/prof_r03b_c4.err
rc=$?; cd $R; [ $rc -eq 0 ] || exit $rc
find gpurun_out/prof_r03b_c4 -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-4 | head -20
