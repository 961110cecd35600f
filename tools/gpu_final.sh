# End-of-iteration check: -m gpu suite, smoke, the default bench line (as the driver runs it: 20 steps,
# 5 warmup, with CPU baseline, parity block and ingest leg), then the C3/C3u/C4/C5 sweep.
# Usage: gpurun -- 'TAG=r02x bash tools/gpu_final.sh'
set -o pipefail
TAG=${TAG:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; python tools/bench_brief.py gpurun_out/bench_$TAG.json; tail -2 gpurun_out/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc
WLS="${WLS:-c3 c3u c4 c5}" TAG=$TAG bash tools/gpu_wls.sh
