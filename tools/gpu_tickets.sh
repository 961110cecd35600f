# GPU tests, then an A/B of the ticket path (TSG_TICKETS=1/0) on the default bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/tk_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/tk_pytest.log; [ $rc -eq 0 ] || exit $rc
STEPS=60 AB="${AB:-TSG_TICKETS=1;TSG_TICKETS=0;TSG_TICKETS=1;TSG_TICKETS=0;TSG_TICKETS=1;TSG_TICKETS=0}" bash tools/gpu_throttle.sh
