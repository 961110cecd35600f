# PMC passes (one counter group per run) over a 1-step bench; per-kernel sums per pass.
# Usage: gpurun -- 'TAG=r02v [BENCH_ARGS="--workload c3"] bash tools/gpu_pmc.sh'
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r02}
cd /tmp
i=0
for g in "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES SQ_WAVES SQ_WAIT_INST_LDS SQ_CYCLES" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g --kernel-trace -d $R/gpurun_out/pmc_${TAG}_$i -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > $R/gpurun_out/pmc_${TAG}_$i.json 2> $R/gpurun_out/pmc_${TAG}_$i.err
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 $R/tools/pmc_summary.py $(find $R/gpurun_out/pmc_${TAG}_$i -name '*counter_collection.csv') > $R/gpurun_out/pmc_${TAG}_$i.txt
  cat $R/gpurun_out/pmc_${TAG}_$i.txt
done
exit 0
