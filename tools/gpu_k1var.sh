# K1 variants: lane chunk 64/128 B x diag modes 0/1/2 at 20 GB (after the GPU tests).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for lane in ${LANES:-64 128}; do
  for m in ${MODES:-0 1 2}; do
    TSG_FILTER_LANE=$lane TSG_DIAG_SCAN=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/var_${lane}_$m.json 2> gpurun_out/var_${lane}_$m.err || exit $?
    python - gpurun_out/var_${lane}_$m.json $lane $m <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read())
print("lane",sys.argv[2],"diag",sys.argv[3],"value",d["value"],"K1",d["breakdown_ms"]["ms_scan_kernel"],"frac",d["roofline"]["frac"],d["breakdown_ms"],d["counts"])
PY
  done
done
if [ -n "${DUMP_GB:-}" ]; then
  TSG_DUMP_CANDS=gpurun_out/cands_${DUMP_GB}g.bin timeout -k 10 300 python bench.py --gb $DUMP_GB --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/dump.json 2> gpurun_out/dump.err || exit $?
  cat gpurun_out/dump.json; ls -la gpurun_out/cands_${DUMP_GB}g.bin
fi
