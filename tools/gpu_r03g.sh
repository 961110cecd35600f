# identity-transformed files read in place: GPU tests (all), C2 bench with the CRLF ingest leg, C4, c1fs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03g}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; python tools/bench_brief.py gpurun_out/bench_$T.json; tail -3 gpurun_out/bench_$T.err; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/bench_$T.json'));print(d['ms_per_step'],d['host_cpu']);i=d['ingest'];print(i['value'],i['ms_per_step'],i['frac_h2d'],i['parity'])"
for wl in c4 c1fs; do
  timeout -k 10 400 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_$wl.json 2> gpurun_out/wl_${T}_$wl.err
  rc=$?; python tools/bench_brief.py gpurun_out/wl_${T}_$wl.json; tail -2 gpurun_out/wl_${T}_$wl.err; [ $rc -eq 0 ] || exit $rc
done
