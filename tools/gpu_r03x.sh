# Final tree: all -m gpu tests, smoke(), three default C2 benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03x}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; tail -1 gpurun_out/smoke_$T.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --ingest-steps 0 > gpurun_out/bench_${T}_$i.json 2> gpurun_out/bench_${T}_$i.err
  rc=$?; python tools/bench_brief.py gpurun_out/bench_${T}_$i.json; [ $rc -eq 0 ] || exit $rc
done
