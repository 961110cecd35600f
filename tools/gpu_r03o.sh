# Round-3 validation: all -m gpu tests, the default bench (driver style), workloads, rocprof
# kernel traces (C2, C4), a FETCH_SIZE pass over C2.  Each step time-limited; stop at a failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${TAG:-r03o}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; python tools/bench_brief.py gpurun_out/bench_$T.json; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/bench_$T.json'));print(d['value'],d['ms_per_step'],d['host_cpu']['process_cpu_ms_per_step'],d['host_cpu']['cpus_used'],(d.get('parity') or {}).get('mismatches'),(d.get('cpu_baseline') or {}).get('value'),(d.get('ingest') or {}).get('value'))"
for wl in c3 c3f c4 c1fs c5; do
  timeout -k 10 500 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${T}_$wl.json 2> gpurun_out/wl_${T}_$wl.err
  rc=$?; echo "== $wl"; python tools/bench_brief.py gpurun_out/wl_${T}_$wl.json; [ $rc -eq 0 ] || exit $rc
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o c2 --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --ingest-steps 0 > $R/gpurun_out/prof_bench_$T.json 2> $R/gpurun_out/prof_$T.err
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4_$T -o c4 --output-format csv -- python3 $R/bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_c4_bench_$T.json 2> $R/gpurun_out/prof_c4_$T.err
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_${T}_fetch -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --ingest-steps 0 > $R/gpurun_out/pmc_${T}_fetch.json 2> $R/gpurun_out/pmc_${T}_fetch.err
rc=$?; echo "fetch pass rc=$rc"; exit $rc
