# SQ counter passes over one C4 step (xform kernels): one group per run
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${TAG:-r03q}
cd /tmp
i=0
for g in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $g --kernel-trace -d $R/gpurun_out/pmc_c4_${T}_$i -o pmc --output-format csv -- python3 $R/bench.py --workload c4 --gb 3 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_c4_${T}_$i.json 2> $R/gpurun_out/pmc_c4_${T}_$i.err
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 $R/tools/pmc_summary.py $(find $R/gpurun_out/pmc_c4_${T}_$i -name '*counter_collection.csv') > $R/gpurun_out/pmc_c4_${T}_$i.txt
  grep -E "xf_|Kernel" $R/gpurun_out/pmc_c4_${T}_$i.txt | cut -c1-250
done
exit 0
