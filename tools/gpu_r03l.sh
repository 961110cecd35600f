# C4 with 2 vs 3 collectors (scans in flight during the walk); analyzer + fs-walk GPU tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03l}
timeout -k 10 300 python -u -m pytest tests/test_analyzer.py tests/test_fs_walk.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
for n in 3 2; do
  timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --collectors $n > gpurun_out/wl_${T}_c4_$n.json 2> gpurun_out/wl_${T}_c4_$n.err
  rc=$?; echo "collectors=$n"; python tools/bench_brief.py gpurun_out/wl_${T}_c4_$n.json; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/wl_${T}_c4_$n.json'));c=d['config'];b=d['breakdown_ms'];print(d['ms_per_step'],d['host_cpu']['cpus_used'],c.get('walk_s_per_step'),c.get('wait_s_per_step'),b['ms_host_gpu_phase'],b['ms_host_exact'])"
done
TSG_WALK_DEBUG=1 timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_c4_dbg.json 2> gpurun_out/wl_${T}_c4_dbg.err
rc=$?; python tools/bench_brief.py gpurun_out/wl_${T}_c4_dbg.json; grep "walk phases" gpurun_out/wl_${T}_c4_dbg.err | tail -1; grep -c "^index" gpurun_out/wl_${T}_c4_dbg.err; exit $rc
