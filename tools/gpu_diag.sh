# K1 diagnostics: timing with/without emission and HBM FETCH_SIZE (separate --pmc pass)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --gb 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/diag_full.json 2>/dev/null || exit $?
TSG_DIAG_SCAN=1 timeout -k 10 600 python bench.py --gb 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/diag_noemit.json 2>/dev/null || exit $?
cd /tmp && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc -o pmc --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --gb 4 --steps 1 --warmup 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/pmc.err
rc=$?; cd $GRAFT_REPO_ROOT; tail -2 gpurun_out/pmc.err; ls gpurun_out/pmc; exit $rc
