# xform identity-tile write path: xform + analyzer GPU tests, C4
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03n}
timeout -k 10 300 python -u -m pytest tests/test_analyzer.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_c4_$i.json 2> gpurun_out/wl_${T}_c4_$i.err
  rc=$?; python tools/bench_brief.py gpurun_out/wl_${T}_c4_$i.json; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/wl_${T}_c4_$i.json'));c=d['config'];b=d['breakdown_ms'];print(d['ms_per_step'],d['host_cpu']['cpus_used'],c.get('walk_s_per_step'),c.get('wait_s_per_step'),b['ms_host_gpu_phase'],b['ms_host_exact'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4_$T -o c4 -- python $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_c4_$T.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; find gpurun_out/prof_c4_$T -name "*kernel_stats.csv" | head -2; exit $rc
