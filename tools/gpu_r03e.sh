# C4 / c1fs after the walk cache: analyzer GPU tests, workloads, walk split, C4 rocprof (xform kernels)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03e}
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_analyzer.py tests/test_fs_walk.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
for wl in c4 c1fs; do
  timeout -k 10 400 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_$wl.json 2> gpurun_out/wl_${T}_$wl.err
  rc=$?; python tools/bench_brief.py gpurun_out/wl_${T}_$wl.json; tail -2 gpurun_out/wl_${T}_$wl.err; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/wl_${T}_$wl.json'));c=d['config'];print(d['ms_per_step'],d['host_cpu'],c.get('walk_s_per_step'),c.get('wait_s_per_step'))"
done
TSG_WALK_DEBUG=1 timeout -k 10 300 python tools/walk_bench.py --gb 4 --reps 2 > gpurun_out/walk_$T.log 2>&1
rc=$?; grep -v "^index:" gpurun_out/walk_$T.log | tail -3; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_c4 -o run --output-format csv -- python3 $R/bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_bench_${T}_c4.json 2> $R/gpurun_out/prof_${T}_c4.err
rc=$?; cd $R; [ $rc -eq 0 ] || exit $rc
find gpurun_out/prof_${T}_c4 -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-4 | cut -c1-120 | head -14
timeout -k 10 400 python tools/k1x.py --gb 20 --reps 5 > gpurun_out/k1x_$T.log 2>&1
rc=$?; cat gpurun_out/k1x_$T.log | tail -30; exit $rc
