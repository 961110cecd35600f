# K2 fire queue by prefix sums, full-scan windows: GPU parity + full-scan tests, C2 A/B of one vs two engine
# slots, C3f
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03h}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_corpus.py tests/test_gpu_fullscan.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
for s in 1 2 1 2; do
  TSG_GPU_SLOTS=$s timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --ingest-steps 0 > gpurun_out/bench_${T}_s$s.json 2> gpurun_out/bench_${T}_s$s.err
  rc=$?; echo "slots=$s"; python tools/bench_brief.py gpurun_out/bench_${T}_s$s.json; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/bench_${T}_s$s.json'));print(d['ms_per_step'],d['host_cpu']['process_cpu_ms_per_step'],d['host_cpu']['cpus_used'],(d.get("parity") or {}).get("mismatches"))"
done
timeout -k 10 400 python bench.py --workload c3f --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_c3f.json 2> gpurun_out/wl_${T}_c3f.err
rc=$?; python tools/bench_brief.py gpurun_out/wl_${T}_c3f.json; tail -2 gpurun_out/wl_${T}_c3f.err; [ $rc -eq 0 ] || exit $rc
for wl in c4; do
  timeout -k 10 400 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_$wl.json 2> gpurun_out/wl_${T}_$wl.err
  rc=$?; python tools/bench_brief.py gpurun_out/wl_${T}_$wl.json; tail -2 gpurun_out/wl_${T}_$wl.err; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/wl_${T}_$wl.json'));c=d['config'];print(d['ms_per_step'],d['host_cpu'],c.get('walk_s_per_step'),c.get('wait_s_per_step'))"
done
TSG_WALK_DEBUG=1 timeout -k 10 300 python tools/walk_bench.py --gb 4 --reps 2 > gpurun_out/walk_$T.log 2>&1
rc=$?; grep -v "^index:" gpurun_out/walk_$T.log | tail -3; exit $rc
