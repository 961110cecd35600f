# K1 iteration: parity, then 4 GB bench in three diag modes, then the 20 GB bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_parity.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_parity.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1 2; do
  TSG_DIAG_SCAN=$m timeout -k 10 600 python bench.py --gb 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/k1_diag$m.json 2> gpurun_out/k1_diag$m.err || exit $?
  echo "diag $m"; cat gpurun_out/k1_diag$m.json
done
timeout -k 10 900 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench20.json 2> gpurun_out/bench20.err
rc=$?; cat gpurun_out/bench20.json; tail -3 gpurun_out/bench20.err; exit $rc
