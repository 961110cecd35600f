# CPU-quota throttling around bench runs: cgroup cpu.stat deltas per setting.
#   gpurun -- 'AB="X=0;TSG_POOL_THREADS=12" bash tools/gpu_throttle.sh'
set -o pipefail
mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.max
IFS=';' read -ra SETS <<< "${AB:-X=0}"
i=0
for s in "${SETS[@]}"; do
  e=${s%%::*}; a=""; [[ "$s" == *::* ]] && a=${s#*::}
  t0=$(grep -E "nr_throttled|throttled_usec|usage_usec" /sys/fs/cgroup/cpu.stat | awk '{print $2}' | tr '\n' ' ')
  env $e timeout -k 10 300 python bench.py --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline --ingest-steps 0 $a > gpurun_out/thr_$i.json 2> gpurun_out/thr_$i.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/thr_$i.err; exit $rc; }
  t1=$(grep -E "nr_throttled|throttled_usec|usage_usec" /sys/fs/cgroup/cpu.stat | awk '{print $2}' | tr '\n' ' ')
  python -c "import json;d=json.load(open('gpurun_out/thr_$i.json'));b=d['breakdown_ms'];a='$t0'.split();z='$t1'.split();print('$s', d['value'], d['ms_per_step'], b['ms_host_gpu_phase'], b['ms_host_exact'], 'cpu_s', (int(z[0])-int(a[0]))/1e6, 'throttled', int(z[1])-int(a[1]), (int(z[2])-int(a[2]))/1e6, 'timed', d.get('host_cpu'))"
  i=$((i+1))
done
