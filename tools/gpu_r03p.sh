# xform one-tile lookahead: xform/analyzer GPU tests, C4 x2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03p}
timeout -k 10 300 python -u -m pytest tests/test_analyzer.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_c4_$i.json 2> gpurun_out/wl_${T}_c4_$i.err
  rc=$?; python tools/bench_brief.py gpurun_out/wl_${T}_c4_$i.json; [ $rc -eq 0 ] || exit $rc
done
