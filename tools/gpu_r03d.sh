# flat xform + pinned path prefilter: xform byte test, GPU parity, analyzer GPU tests, C2 A/B, C4 / c1fs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03d}
timeout -k 10 300 python -u -m pytest tests/test_analyzer.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  TSG_GPU_ALLOW_PATH=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --ingest-steps 0 > gpurun_out/bench_${T}_ap$v.json 2> gpurun_out/bench_${T}_ap$v.err
  rc=$?; echo "allow-path gpu=$v"; python tools/bench_brief.py gpurun_out/bench_${T}_ap$v.json; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/bench_${T}_ap$v.json'));print(d['ms_per_step'],d['host_cpu'],{k:v for k,v in d['breakdown_ms'].items() if 'host' in k})"
done
for wl in c4 c1fs; do
  timeout -k 10 400 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_$wl.json 2> gpurun_out/wl_${T}_$wl.err
  rc=$?; python tools/bench_brief.py gpurun_out/wl_${T}_$wl.json; tail -2 gpurun_out/wl_${T}_$wl.err; [ $rc -eq 0 ] || exit $rc
done
TSG_WALK_DEBUG=1 timeout -k 10 300 python tools/walk_bench.py --gb 4 --reps 2 > gpurun_out/walk_$T.log 2>&1
rc=$?; grep -v "^index:" gpurun_out/walk_$T.log | tail -4; [ $rc -eq 0 ] || exit $rc
