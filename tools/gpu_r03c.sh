# allow-path GPU prefilter check: its parity test, the GPU parity suite, C2 A/B (prefilter on / off)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03c}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  TSG_GPU_ALLOW_PATH=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --ingest-steps 0 > gpurun_out/bench_${T}_ap$v.json 2> gpurun_out/bench_${T}_ap$v.err
  rc=$?; echo "allow-path gpu=$v"; python tools/bench_brief.py gpurun_out/bench_${T}_ap$v.json; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/bench_${T}_ap$v.json'));print(d['ms_per_step'],d['host_cpu'])"
done
