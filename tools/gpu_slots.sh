# GPU tests, then the default bench with 1 / 2 GPU slots (TSG_GPU_SLOTS) at depths 3 and 4.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-1:3 2:3 2:4}; do
  sl=${cfg%%:*}; d=${cfg##*:}
  TSG_GPU_SLOTS=$sl timeout -k 10 300 python bench.py --steps 8 --warmup 2 --depth $d --no-cpu-baseline > gpurun_out/bench_s${sl}d$d.json 2> gpurun_out/bench_s${sl}d$d.err
  rc=$?; echo "== slots $sl depth $d"; python -c "import json,sys;j=json.load(open(sys.argv[1]));print(j['value'],j['ms_per_step'],j['roofline']['achieved'],j['breakdown_ms'])" gpurun_out/bench_s${sl}d$d.json; tail -2 gpurun_out/bench_s${sl}d$d.err; [ $rc -eq 0 ] || exit $rc
done
