# Profile set for the committed build: rocprofv3 kernel-trace stats and FETCH_SIZE (PMC) passes of
# the default C2 bench and of C3, plus one SQ pass per workload on the dominant kernels.
# Usage: gpurun -- 'TAG=r02x bash tools/gpu_profiles.sh'
set -o pipefail
TAG=${TAG:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
prof() {  # name, args...
  local n=$1; shift
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_$n -o run --output-format csv -- python3 $R/bench.py "$@" > $R/gpurun_out/prof_${TAG}_$n.json 2> $R/gpurun_out/prof_${TAG}_$n.err
  local rc=$?; cd $R; echo "== prof $n rc=$rc"; [ $rc -eq 0 ] || return $rc
  python3 tools/bench_brief.py gpurun_out/prof_${TAG}_$n.json
  find gpurun_out/prof_${TAG}_$n -name '*kernel_stats.csv' -exec head -9 {} \;
}
pmc() {  # name, counters, args...
  local n=$1 ctr=$2; shift 2
  cd /tmp
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace -d $R/gpurun_out/pmc_${TAG}_$n -o pmc --output-format csv -- python3 $R/bench.py "$@" > $R/gpurun_out/pmc_${TAG}_$n.json 2> $R/gpurun_out/pmc_${TAG}_$n.err
  local rc=$?; cd $R; echo "== pmc $n rc=$rc"; return $rc
}
prof c2 --steps 3 --warmup 1 --no-cpu-baseline --ingest-steps 0 &&
prof c3 --workload c3 --steps 3 --warmup 1 --no-cpu-baseline &&
pmc c2_fetch FETCH_SIZE --steps 1 --warmup 0 --no-cpu-baseline --ingest-steps 0 &&
pmc c3_fetch FETCH_SIZE --workload c3 --steps 1 --warmup 0 --no-cpu-baseline &&
pmc c2_sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY" --steps 1 --warmup 0 --no-cpu-baseline --ingest-steps 0 &&
pmc c3_sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY" --workload c3 --steps 1 --warmup 0 --no-cpu-baseline
