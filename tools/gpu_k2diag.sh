# K2 (confirm) diag sweep at 20 GB: TSG_DIAG_CONFIRM bits 4 (fires only), 1|2 (no NFA, no line count), 2, 0
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in ${DIAGS:-4 3 2 0}; do
  TSG_STATS_DEBUG=1 TSG_DIAG_CONFIRM=$d timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/k2d_$d.json 2> gpurun_out/k2d_$d.err || exit $?
  python - gpurun_out/k2d_$d.json $d <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read())
import subprocess
print(open(sys.argv[1].replace(".json",".err")).read()[-300:])
print("confirm diag",sys.argv[2],"K1",d["breakdown_ms"]["ms_scan_kernel"],"K2",d["breakdown_ms"]["ms_verify_kernel"],"careful",d["breakdown_ms"]["ms_careful_kernel"],d["counts"])
PY
done
