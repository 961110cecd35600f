# Workload sweep on one box: C2 as the driver runs it (20 steps, 5 warmup), C3, C3u, C4, C5.
# Usage: gpurun -- 'TAG=r02x bash tools/gpu_wls.sh'
set -o pipefail
TAG=${TAG:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > gpurun_out/wl_${TAG}_$n.json 2> gpurun_out/wl_${TAG}_$n.err
  local rc=$?; echo "== $n rc=$rc"; python tools/bench_brief.py gpurun_out/wl_${TAG}_$n.json; tail -2 gpurun_out/wl_${TAG}_$n.err; return $rc
}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for w in ${WLS:-c2 c3 c3u c4 c5}; do
  case $w in
    c2) run c2 400 --steps 20 --warmup 5 --no-cpu-baseline --ingest-steps 0 ;;
    c3) run c3 400 --workload c3 --steps 5 --warmup 1 ;;
    c3u) run c3u 400 --workload c3u --steps 5 --warmup 1 --no-cpu-baseline ;;
    c3u0) TSG_CLASS_RUNS=0 run c3u0 400 --workload c3u --steps 3 --warmup 1 --no-cpu-baseline ;;
    c3h0) TSG_WINDOW_HASH=0 run c3h0 400 --workload c3 --steps 5 --warmup 1 --no-cpu-baseline ;;
    c3f0) TSG_FOLD_INDEX=0 run c3f0 400 --workload c3 --steps 5 --warmup 1 --no-cpu-baseline ;;
    c2h0) TSG_WINDOW_HASH=0 run c2h0 400 --steps 20 --warmup 5 --no-cpu-baseline --ingest-steps 0 ;;
    c4) run c4 500 --workload c4 --steps 3 --warmup 1 --no-cpu-baseline ;;
    c5) run c5 500 --workload c5 --steps 2 --warmup 1 --pool-gb 32 --no-cpu-baseline ;;
  esac || exit $?
done
