# K1 without the in-loop scratch reload; confirm next-record prefetch -- parity tests, C2 x3
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03u}
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_corpus.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --ingest-steps 0 > gpurun_out/bench_${T}_$i.json 2> gpurun_out/bench_${T}_$i.err
  rc=$?; python tools/bench_brief.py gpurun_out/bench_${T}_$i.json; [ $rc -eq 0 ] || exit $rc
done
