# C4 after the index changes; pool size A/B; walk bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03m}
for cfg in "def" "15" "def"; do
  if [ "$cfg" = def ]; then unset TSG_POOL_THREADS; else export TSG_POOL_THREADS=$cfg; fi
  timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_c4_$cfg.json 2> gpurun_out/wl_${T}_c4_$cfg.err
  rc=$?; echo "pool=$cfg"; python tools/bench_brief.py gpurun_out/wl_${T}_c4_$cfg.json; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/wl_${T}_c4_$cfg.json'));c=d['config'];b=d['breakdown_ms'];print(d['ms_per_step'],d['host_cpu']['cpus_used'],c.get('walk_s_per_step'),c.get('wait_s_per_step'),b['ms_host_gpu_phase'],b['ms_host_exact'])"
done
unset TSG_POOL_THREADS
TSG_WALK_DEBUG=1 timeout -k 10 200 python tools/walk_bench.py --gb 4 --reps 3 > gpurun_out/walk_${T}.log 2>&1
rc=$?; grep -v "^index" gpurun_out/walk_${T}.log | tail -2; grep "^index" gpurun_out/walk_${T}.log | tail -2; exit $rc
