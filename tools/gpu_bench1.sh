set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --gb 2 --steps 3 --warmup 1 --cpu-sample-mb 8 > gpurun_out/bench_2g.json 2> gpurun_out/bench_2g.err
rc=$?
cat gpurun_out/bench_2g.json; tail -5 gpurun_out/bench_2g.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_20g.json 2> gpurun_out/bench_20g.err
rc=$?
cat gpurun_out/bench_20g.json; tail -5 gpurun_out/bench_20g.err
exit $rc
