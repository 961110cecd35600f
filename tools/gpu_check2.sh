# GPU tests, then N default-bench runs (no CPU baseline) with the timed-region CPU use.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c2_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/c2_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq 1 ${RUNS:-3}); do
  env ${ENVS:-X=0} timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --ingest-steps 0 ${ARGS:-} > gpurun_out/c2_b$i.json 2> gpurun_out/c2_b$i.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/c2_b$i.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/c2_b$i.json'));b=d['breakdown_ms'];print(d['value'], d['ms_per_step'], b['ms_gpu_total'], b['ms_host_gpu_phase'], b['ms_host_exact'], d.get('host_cpu'), (d.get('parity') or {}).get('mismatches'))"
done
