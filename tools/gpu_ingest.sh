# Ingest-inclusive C2 bench (--ingest) + a kernel/memcpy trace of the same for copy/kernel overlap.
# Usage: gpurun -- 'TAG=r02g bash tools/gpu_ingest.sh'
set -o pipefail
TAG=${TAG:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py --ingest --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ingest_$TAG.json 2> gpurun_out/bench_ingest_$TAG.err
rc=$?; cat gpurun_out/bench_ingest_$TAG.json; tail -3 gpurun_out/bench_ingest_$TAG.err; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/trace_ingest_$TAG -o run --output-format csv -- python3 $R/bench.py --ingest --steps 1 --warmup 0 --no-cpu-baseline --gb 8 > $R/gpurun_out/trace_ingest_bench_$TAG.json 2> $R/gpurun_out/trace_ingest_$TAG.err
rc=$?; cd $R; tail -2 gpurun_out/trace_ingest_$TAG.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload c3 --steps 5 --warmup 1 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err
rc=$?; cat gpurun_out/bench_c3_$TAG.json; tail -3 gpurun_out/bench_c3_$TAG.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
rc=$?; cat gpurun_out/bench_c4_$TAG.json; tail -3 gpurun_out/bench_c4_$TAG.err; exit $rc
