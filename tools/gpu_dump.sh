# dump GPU candidates of the 4 GB bench corpus (host-tail profiling on CPU) + a kernel-trace profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TSG_DUMP_CANDS=$GRAFT_REPO_ROOT/gpurun_out/cands_4g.bin timeout -k 10 600 python bench.py --gb 4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/dump.json 2> gpurun_out/dump.err || exit $?
ls -la gpurun_out/cands_4g.bin
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --gb 20 --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err
rc=$?; cd $GRAFT_REPO_ROOT; tail -2 gpurun_out/prof.err; find gpurun_out/prof -name '*stats*'; exit $rc
