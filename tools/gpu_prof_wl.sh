# rocprofv3 kernel-trace stats of the c3 / c4 workloads (small sizes).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${TAG:-wl}
for wl in ${WLS:-c3 c4}; do
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_$wl -o run --output-format csv -- python3 $R/bench.py --workload $wl --gb ${GB:-4} --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_${TAG}_$wl.json 2> $R/gpurun_out/prof_${TAG}_$wl.err
  rc=$?; cd $R; tail -2 gpurun_out/prof_${TAG}_$wl.err; [ $rc -eq 0 ] || exit $rc
  cat gpurun_out/prof_${TAG}_$wl.json
  find gpurun_out/prof_${TAG}_$wl -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-4
done
