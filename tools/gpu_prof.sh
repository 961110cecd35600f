# Kernel-trace stats of a 4 GB bench + SQ PMC passes on K1 (diag 0 and 1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r01x}
GB=${GB:-4}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --gb $GB --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err
rc=$?; cd $R; tail -2 gpurun_out/prof.err; [ $rc -eq 0 ] || exit $rc
cat gpurun_out/prof_bench.json
find gpurun_out/prof_$TAG -name '*kernel_stats.csv' -exec cat {} \;
for m in ${PMC_MODES:-1 0}; do
  cd /tmp
  TSG_DIAG_SCAN=$m timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d $R/gpurun_out/pmc_sq$m -o pmc --output-format csv -- python3 $R/bench.py --gb $GB --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_sq$m.json 2> $R/gpurun_out/pmc_sq$m.err
  rc=$?; cd $R; tail -2 gpurun_out/pmc_sq$m.err; [ $rc -eq 0 ] || exit $rc
  python3 - gpurun_out/pmc_sq$m <<'PY'
import csv, glob, sys, collections
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if __import__("os").environ.get("KNAME", "filter_kernel") in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(sys.argv[1], dict(agg))
PY
done
