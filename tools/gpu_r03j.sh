# C4 walk anatomy on the box: C4 bench with the walk's phase timers, walk bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03j}
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python -c "import os; print(len(os.sched_getaffinity(0)))"
TSG_WALK_DEBUG=1 timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_c4.json 2> gpurun_out/wl_${T}_c4.err
rc=$?; python tools/bench_brief.py gpurun_out/wl_${T}_c4.json; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/wl_${T}_c4.json'));c=d['config'];print(d['ms_per_step'],d['host_cpu'],c.get('walk_s_per_step'),c.get('wait_s_per_step'))"
grep "walk phases" gpurun_out/wl_${T}_c4.err | tail -1
for i in 1 2; do
  TSG_WALK_DEBUG=1 timeout -k 10 200 python tools/walk_bench.py --gb 4 --reps 2 > gpurun_out/walk_${T}_$i.log 2>&1
  rc=$?; grep -v "^index:" gpurun_out/walk_${T}_$i.log | tail -2; [ $rc -eq 0 ] || exit $rc
done
