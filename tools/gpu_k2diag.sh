# Confirm-kernel cost split (TSG_DIAG_CONFIRM modes) at C2, 20 GB, 3 steps each:
#   0 full; 4 phase A only (fires not queued); 16 phase B + item sets, no attribution;
#   8 attribution, no emission.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in ${DIAGS:-0 4 16 8}; do
  TSG_DIAG_CONFIRM=$d timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/k2diag_$d.json 2> gpurun_out/k2diag_$d.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/k2diag_$d.json'));b=d['breakdown_ms'];c=d['counts'];print('diag $d', b['ms_scan_kernel'], b['ms_confirm_kernel'], b['ms_nfa_kernel'], b['ms_gpu_total'], c['anchor_hits'], c['candidates'])"
done
