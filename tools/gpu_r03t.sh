# Final round-3 check on the box: all -m gpu tests, smoke(), the default bench (driver-style), rocprof kernel
# stats of the default C2 bench.  Each step time-limited; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${TAG:-r03t}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; python tools/bench_brief.py gpurun_out/bench_$T.json; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/bench_$T.json'));print(d['value'],d['steps'],d['ms_per_step'],d['host_cpu']['process_cpu_ms_per_step'],d['host_cpu']['cpus_used'],(d.get('parity') or {}).get('mismatches'),(d.get('cpu_baseline') or {}).get('value'),(d.get('ingest') or {}).get('value'),d['roofline']['frac'],d['roofline'].get('k1',{}).get('frac'))"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o c2 --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --ingest-steps 0 > $R/gpurun_out/prof_bench_$T.json 2> $R/gpurun_out/prof_$T.err
rc=$?; echo "prof rc=$rc"; exit $rc
