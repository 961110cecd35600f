# xform rewrite (segments, masks) + C2 with 5% CRLF: xform/analyzer GPU tests, C2 bench (CRLF, ingest leg
# strips on the GPU), C4 + c1fs, C4 rocprof
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03f}
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_analyzer.py tests/test_fs_walk.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-sample-mb 200 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; python tools/bench_brief.py gpurun_out/bench_$T.json; tail -3 gpurun_out/bench_$T.err; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/bench_$T.json'));print(d['ms_per_step'],d['host_cpu'],d['ingest'],d['parity'],d['config'])"
for wl in c4 c1fs; do
  timeout -k 10 400 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_$wl.json 2> gpurun_out/wl_${T}_$wl.err
  rc=$?; python tools/bench_brief.py gpurun_out/wl_${T}_$wl.json; tail -2 gpurun_out/wl_${T}_$wl.err; [ $rc -eq 0 ] || exit $rc
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_c4 -o run --output-format csv -- python3 $R/bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_bench_${T}_c4.json 2> $R/gpurun_out/prof_${T}_c4.err
rc=$?; cd $R; [ $rc -eq 0 ] || exit $rc
find gpurun_out/prof_${T}_c4 -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-4 | cut -c1-110 | head -8
