# Final check: smoke(), GPU tests, then a host-thread / depth sweep of the default bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-16:3 24:3 16:4 12:3}; do
  th=${cfg%%:*}; d=${cfg##*:}
  TSG_HOST_THREADS=$th timeout -k 10 300 python bench.py --steps 8 --warmup 2 --depth $d --no-cpu-baseline > gpurun_out/bench_t${th}d$d.json 2> gpurun_out/bench_t${th}d$d.err
  rc=$?; echo "== threads $th depth $d"; python -c "import json,sys;j=json.load(open(sys.argv[1]));print(j['value'],j['ms_per_step'],j['breakdown_ms'])" gpurun_out/bench_t${th}d$d.json; [ $rc -eq 0 ] || exit $rc
done
