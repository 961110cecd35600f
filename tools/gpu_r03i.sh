# Full scan boundary pass: full-scan + parity tests, C3f; walk A/B (index window), path views; C4
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03i}
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullscan.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload c3f --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_c3f.json 2> gpurun_out/wl_${T}_c3f.err
rc=$?; python tools/bench_brief.py gpurun_out/wl_${T}_c3f.json; tail -2 gpurun_out/wl_${T}_c3f.err; [ $rc -eq 0 ] || exit $rc
for ah in 8 2 8; do
  TSG_WALK_AHEAD=$ah TSG_WALK_DEBUG=1 timeout -k 10 200 python tools/walk_bench.py --gb 4 --reps 2 > gpurun_out/walk_${T}_$ah.log 2>&1
  rc=$?; echo "ahead=$ah"; grep -v "^index:" gpurun_out/walk_${T}_$ah.log | tail -2; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_c4.json 2> gpurun_out/wl_${T}_c4.err
rc=$?; python tools/bench_brief.py gpurun_out/wl_${T}_c4.json; tail -2 gpurun_out/wl_${T}_c4.err; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/wl_${T}_c4.json'));c=d['config'];print(d['ms_per_step'],d['host_cpu'],c.get('walk_s_per_step'),c.get('wait_s_per_step'))"
