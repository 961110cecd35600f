# Round measurement: GPU parity, the default bench (20 GB, with cpu_baseline), K1 diag modes,
# a rocprofv3 kernel-trace/stats pass and a separate FETCH_SIZE (PMC) pass of the same workload.
# Usage: gpurun -- 'bash tools/gpu_full.sh'   (TAG=r01 by default)
set -o pipefail
TAG=${TAG:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
if [ -n "${DIAG:-}" ]; then
  for m in 1 2; do
    TSG_DIAG_SCAN=$m timeout -k 10 300 python bench.py --gb 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/k1_diag$m.json 2> gpurun_out/k1_diag$m.err || exit $?
    echo "diag $m"; cat gpurun_out/k1_diag$m.json
  done
fi
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err
rc=$?; cd $R; tail -2 gpurun_out/prof.err; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_$TAG -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_bench.json 2> $R/gpurun_out/pmc.err
rc=$?; cd $R; tail -2 gpurun_out/pmc.err; find gpurun_out/prof_$TAG gpurun_out/pmc_$TAG -name '*.csv' | head -20; exit $rc
