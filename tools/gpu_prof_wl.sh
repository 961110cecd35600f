# rocprof kernel stats of one bench workload: WL=c4 TAG=r03c bash tools/gpu_prof_wl.sh
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
for wl in ${WLS:-c4}; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_$wl -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --ingest-steps 0 ${EXTRA:-} > $R/gpurun_out/prof_${TAG}_$wl.json 2> $R/gpurun_out/prof_${TAG}_$wl.err
  rc=$?; tail -2 $R/gpurun_out/prof_${TAG}_$wl.err; [ $rc -eq 0 ] || exit $rc
  find $R/gpurun_out/prof_${TAG}_$wl -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-8 | head -16
done
