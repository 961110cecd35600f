# GPU iteration runner (rounds 5-6): stages chosen by STAGES (space-separated), each under its own time limit,
# stopping at the first failure.  Usage: gpurun -- 'TAG=r04a STAGES="tests bench diag prof" bash tools/gpu_run.sh'
#   tests  : the -m gpu suite (PYTEST_K: a -k expression; PYTEST_ARGS: more words)
#   smoke  : __graft_entry__.smoke()
#   bench  : the driver-style default line (20 steps, 5 warm-up, CPU baseline, parity, ingest leg)
#   quick  : C2 without the CPU baseline (BENCH_ARGS adds flags)
#   diag   : C2 confirm-kernel split (TSG_DIAG_CONFIRM 4 / 8 / 16), 5 steps each
#   prof   : rocprofv3 --kernel-trace --stats of a short C2 run
#   wl     : the workloads in WLS (default c3 c3f c4 c1fs c5), with CPU baselines unless WL_ARGS says otherwise;
#            WL_ARGS_<wl> adds flags for one workload
set -o pipefail
TAG=${TAG:-r05}
STAGES=${STAGES:-tests bench}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for st in $STAGES; do
  case $st in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS:-} > gpurun_out/gpu_tests_$TAG.log 2>&1
      rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
      rc=$?; tail -2 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
      rc=$?; python tools/bench_brief.py gpurun_out/bench_$TAG.json; tail -2 gpurun_out/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc ;;
    dflt)  # the default bench (no flags), DFLT_N times
      for i in $(seq 1 ${DFLT_N:-2}); do
        timeout -k 10 600 python bench.py > gpurun_out/dflt_${TAG}_$i.json 2> gpurun_out/dflt_${TAG}_$i.err
        rc=$?; echo "== default $i"; python tools/bench_brief.py gpurun_out/dflt_${TAG}_$i.json; tail -1 gpurun_out/dflt_${TAG}_$i.err; [ $rc -eq 0 ] || exit $rc
      done ;;
    quick)
      timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/quick_$TAG.json 2> gpurun_out/quick_$TAG.err
      rc=$?; python tools/bench_brief.py gpurun_out/quick_$TAG.json; tail -2 gpurun_out/quick_$TAG.err; [ $rc -eq 0 ] || exit $rc ;;
    diag)
      for d in 0 4 8 16; do
        TSG_DIAG_CONFIRM=$d timeout -k 10 300 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --ingest-steps 0 ${BENCH_ARGS:-} > gpurun_out/diag${d}_$TAG.json 2> gpurun_out/diag${d}_$TAG.err
        rc=$?; echo "== diag $d"; python tools/bench_brief.py gpurun_out/diag${d}_$TAG.json; [ $rc -eq 0 ] || exit $rc
      done ;;
    prof)
      cd /tmp
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --ingest-steps 0 > $R/gpurun_out/prof_bench_$TAG.json 2> $R/gpurun_out/prof_$TAG.err
      rc=$?; cd $R; tail -2 gpurun_out/prof_$TAG.err; [ $rc -eq 0 ] || exit $rc
      find gpurun_out/prof_$TAG -name '*kernel_stats.csv' -exec cat {} \; ;;
    c4prof)  # rocprofv3 kernel stats of a short C4 run (the pre-transform kernels per batch)
      cd /tmp
      timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c4prof_$TAG -o run --output-format csv -- python3 $R/bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline ${C4PROF_ARGS:-} > $R/gpurun_out/c4prof_bench_$TAG.json 2> $R/gpurun_out/c4prof_$TAG.err
      rc=$?; cd $R; tail -2 gpurun_out/c4prof_$TAG.err; [ $rc -eq 0 ] || exit $rc
      find gpurun_out/c4prof_$TAG -name '*kernel_stats.csv' -exec cat {} \; ;;
    ingprof)  # the C2 ingest leg under a kernel + memory-copy trace (copy / kernel timeline)
      cd /tmp
      timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/ingprof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --warmup-s 0 --no-cpu-baseline --ingest-steps 3 > $R/gpurun_out/ingprof_bench_$TAG.json 2> $R/gpurun_out/ingprof_$TAG.err
      rc=$?; cd $R; tail -2 gpurun_out/ingprof_$TAG.err; [ $rc -eq 0 ] || exit $rc
      python tools/bench_brief.py gpurun_out/ingprof_bench_$TAG.json ;;
    ab)  # C2 A/B of library variants (VARIANTS="base pf ..."; base = the in-tree build), twice interleaved
      for rep in 1 2; do
        for v in ${VARIANTS:-base}; do
          if [ "$v" = base ]; then L=""; else L=$R/trivy_amd/_variants/$v/libtsg.so; fi
          TSG_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ingest-steps 0 ${BENCH_ARGS:-} > gpurun_out/ab_${TAG}_${v}_$rep.json 2> gpurun_out/ab_${TAG}_${v}_$rep.err
          rc=$?; echo "== $v $rep"; python tools/bench_brief.py gpurun_out/ab_${TAG}_${v}_$rep.json; [ $rc -eq 0 ] || exit $rc
        done
      done ;;
    dump)  # candidates of one C3f scan for tools/host_tail_bench.py (CPU profiling of the exact pass)
      TSG_TAIL_DEBUG=1 TSG_DUMP_CANDS=$R/gpurun_out/cands_${DUMP_WL:-c3f}.bin timeout -k 10 600 python bench.py --workload ${DUMP_WL:-c3f} --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/dump_$TAG.json 2> gpurun_out/dump_$TAG.err
      rc=$?; ls -la gpurun_out/cands_${DUMP_WL:-c3f}.bin; grep -a "tail" gpurun_out/dump_$TAG.err | tail -4; [ $rc -eq 0 ] || exit $rc ;;
    k1x)  # the K1 inner-loop experiments (tools/k1x.hip, built in-tree beforehand), K1X_ONLY: variant indices
      timeout -k 10 400 python tools/k1x.py --gb ${K1X_GB:-20} --reps 5 ${K1X_ONLY:+--only $K1X_ONLY} > gpurun_out/k1x_$TAG.log 2>&1
      rc=$?; cat gpurun_out/k1x_$TAG.log | grep -v "^$" | tail -40; [ $rc -eq 0 ] || exit $rc ;;
    k1xpmc)  # SQ counters of chosen k1x variants (one --pmc pass per counter set)
      cd /tmp
      for v in ${K1X_ONLY:-19}; do
        timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES -d $R/gpurun_out/k1xpmc_${TAG}_$v -o run --output-format csv -- python3 $R/tools/k1x.py --gb ${K1X_GB:-20} --reps 1 --only $v > $R/gpurun_out/k1xpmc_${TAG}_$v.log 2>&1
        rc=$?; [ $rc -eq 0 ] || { cd $R; tail -5 gpurun_out/k1xpmc_${TAG}_$v.log; exit $rc; }
      done
      cd $R ;;
    c4l)  # C4 under several bench arg sets (C4L_SPECS, '|'-separated), e.g. "--layers 1|--layers 5 --layer-parallel 3"
      IFS='|' read -r -a specs <<< "${C4L_SPECS:---layers 1}"
      for i in "${!specs[@]}"; do
        timeout -k 10 600 python bench.py --workload c4 --steps ${C4_STEPS:-5} --warmup 2 --no-cpu-baseline ${specs[$i]} > gpurun_out/c4l_${TAG}_$i.json 2> gpurun_out/c4l_${TAG}_$i.err
        rc=$?; echo "== c4 [$i] ${specs[$i]}"; python tools/bench_brief.py gpurun_out/c4l_${TAG}_$i.json; [ $rc -eq 0 ] || exit $rc
      done ;;
    walkprof)  # the C4 tar walk alone on the box's host cores (no GPU), with the sampling profiler
      SPROF=$R/gpurun_out/walkprof_$TAG.txt TSG_WALK_DEBUG=1 timeout -k 10 600 python tools/walk_bench.py --gb ${WALK_GB:-15} --reps 3 > gpurun_out/walkprof_$TAG.log 2>&1
      rc=$?; grep -v "^index:" gpurun_out/walkprof_$TAG.log | tail -4; [ $rc -eq 0 ] || exit $rc
      python tools/sprof/report.py gpurun_out/walkprof_$TAG.txt libtsg_host > gpurun_out/walkprof_${TAG}_fn.txt 2>&1
      python tools/sprof/report.py gpurun_out/walkprof_$TAG.txt libtsg_host lines > gpurun_out/walkprof_${TAG}_lines.txt 2>&1
      head -30 gpurun_out/walkprof_${TAG}_fn.txt ;;
    tailprof)  # the exact host pass on the box's cores over a dumped candidate list (TAIL_CANDS, TAIL_WL)
      TSG_TAIL_DEBUG=1 timeout -k 10 600 python tools/host_tail_bench.py ${TAIL_CANDS} --workload ${TAIL_WL:-c2} --gb ${TAIL_GB:-20} --reps 5 > gpurun_out/tailprof_$TAG.log 2>&1
      rc=$?; grep "serial\|tail \|phases" gpurun_out/tailprof_$TAG.log | tail -6; [ $rc -eq 0 ] || exit $rc ;;
    dumps)  # candidates of one C2 and one C3f scan (tools/host_tail_bench.py)
      for wl in c2 c3f; do
        TSG_DUMP_CANDS=$R/gpurun_out/cands_${wl}_$TAG.bin timeout -k 10 600 python bench.py --workload $wl --steps 1 --warmup 0 --warmup-s 0 --ingest-steps 0 --no-cpu-baseline > gpurun_out/dump_${wl}_$TAG.json 2> gpurun_out/dump_${wl}_$TAG.err
        rc=$?; ls -la gpurun_out/cands_${wl}_$TAG.bin; [ $rc -eq 0 ] || exit $rc
      done ;;
    large)  # the > 4 GiB transformed-file test alone (last: it moves ~9 GB through the box)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_large_file.py -x -q --timeout 500 --timeout-method thread > gpurun_out/gpu_large_$TAG.log 2>&1
      rc=$?; tail -3 gpurun_out/gpu_large_$TAG.log; [ $rc -eq 0 ] || exit $rc ;;
    abenv)  # C2 A/B over "variant[:ENV=V ...]" specs ('|'-separated AB_SPECS; variant base = the in-tree build), twice interleaved
      IFS='|' read -r -a specs <<< "${AB_SPECS:-base}"
      for rep in 1 2; do
        for i in "${!specs[@]}"; do
          sp="${specs[$i]}"; v="${sp%%:*}"; E=""; [ "$sp" != "$v" ] && E="${sp#*:}"
          if [ "$v" = base ]; then L=""; else L=$R/trivy_amd/_variants/$v/libtsg.so; fi
          env TSG_LIB=$L $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ingest-steps 0 ${BENCH_ARGS:-} > gpurun_out/abenv_${TAG}_${i}_$rep.json 2> gpurun_out/abenv_${TAG}_${i}_$rep.err
          rc=$?; echo "== [$i] $sp $rep"; python tools/bench_brief.py gpurun_out/abenv_${TAG}_${i}_$rep.json; [ $rc -eq 0 ] || exit $rc
        done
      done ;;
    ingab)  # ingest leg A/B of library variants (VARIANTS; base = the in-tree build), twice interleaved
      for rep in 1 2; do
        for sp in ${VARIANTS:-base}; do  # variant[:ENV=V] (one env assignment)
          v="${sp%%:*}"; E=""; [ "$sp" != "$v" ] && E="${sp#*:}"
          if [ "$v" = base ]; then L=""; else L=$R/trivy_amd/_variants/$v/libtsg.so; fi
          v="$v${E:+_${E//=/}}"
          env TSG_LIB=$L $E timeout -k 10 400 python bench.py --steps 5 --warmup 2 --warmup-s 0 --no-cpu-baseline --ingest-steps ${INGEST_STEPS:-6} ${BENCH_ARGS:-} > gpurun_out/ingab_${TAG}_${v}_$rep.json 2> gpurun_out/ingab_${TAG}_${v}_$rep.err
          rc=$?; echo "== $v $rep"; python - gpurun_out/ingab_${TAG}_${v}_$rep.json <<'PYEOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
i = d.get("ingest") or {}
print("value=%s ingest=%s frac_h2d=%s ms=%s" % (d["value"], i.get("value"), i.get("frac_h2d"), i.get("ms_per_step")))
PYEOF
          [ $rc -eq 0 ] || exit $rc
        done
      done ;;
    c4ab)  # C4 with the defaults and with each env of C4_ENVS ('|'-separated, e.g. "TSG_INGEST_CHUNK_MB=64|TSG_GPU_SLOTS=2"), interleaved
      IFS='|' read -r -a envs <<< "${C4_ENVS:-TSG_INGEST_CHUNK_MB=64}"
      for rep in 1 2; do
        for i in base "${!envs[@]}"; do
          if [ "$i" = base ]; then E=""; v=base; else E="${envs[$i]}"; v=alt$i; fi
          env $E timeout -k 10 600 python bench.py --workload c4 --steps ${C4_STEPS:-5} --warmup 2 --no-cpu-baseline ${C4_ARGS:-} > gpurun_out/c4ab_${TAG}_${v}_$rep.json 2> gpurun_out/c4ab_${TAG}_${v}_$rep.err
          rc=$?; echo "== c4 $v $rep ($E)"; python tools/bench_brief.py gpurun_out/c4ab_${TAG}_${v}_$rep.json; [ $rc -eq 0 ] || exit $rc
        done
      done ;;
    pmc)  # SQ counters per kernel, two passes (tools/gpu_pmc.sh groups 1-2) over a 1-step C2 run
      cd /tmp
      i=0
      for g in "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES SQ_WAVES SQ_WAIT_INST_LDS SQ_CYCLES" \
               "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD"; do
        i=$((i+1))
        timeout -s KILL 150 rocprofv3 --pmc $g --kernel-trace -d $R/gpurun_out/pmc_${TAG}_$i -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --warmup-s 0 --no-cpu-baseline --ingest-steps 0 ${BENCH_ARGS:-} > $R/gpurun_out/pmc_${TAG}_$i.json 2> $R/gpurun_out/pmc_${TAG}_$i.err
        rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
        python3 $R/tools/pmc_summary.py $(find $R/gpurun_out/pmc_${TAG}_$i -name '*counter_collection.csv') > $R/gpurun_out/pmc_${TAG}_$i.txt
        cat $R/gpurun_out/pmc_${TAG}_$i.txt
      done
      cd $R ;;
    fetch)  # HBM traffic: FETCH_SIZE and WRITE_SIZE, one pass each, over a 1-step run (BENCH_ARGS picks the workload)
      cd /tmp
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/fetch_${TAG}_$c -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --warmup-s 0 --no-cpu-baseline --ingest-steps 0 ${BENCH_ARGS:-} > $R/gpurun_out/fetch_${TAG}_$c.json 2> $R/gpurun_out/fetch_${TAG}_$c.err
        rc=$?; echo "pass $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
        python3 $R/tools/pmc_summary.py $(find $R/gpurun_out/fetch_${TAG}_$c -name '*counter_collection.csv') > $R/gpurun_out/fetch_${TAG}_$c.txt
        cat $R/gpurun_out/fetch_${TAG}_$c.txt
      done
      cd $R ;;
    runs)  # bench lines RUNS="name:args|name:args" (each its own time limit), e.g. "c3f6:--workload c3f --depth 6"
      IFS='|' read -r -a rs <<< "${RUNS}"
      for r in "${rs[@]}"; do
        n="${r%%:*}"; a="${r#*:}"
        timeout -k 10 600 python bench.py $a > gpurun_out/run_${TAG}_$n.json 2> gpurun_out/run_${TAG}_$n.err
        rc=$?; echo "== $n ($a)"; python tools/bench_brief.py gpurun_out/run_${TAG}_$n.json; tail -1 gpurun_out/run_${TAG}_$n.err; [ $rc -eq 0 ] || exit $rc
      done ;;
    wl)
      for wl in ${WLS:-c3 c3f c4 c1fs c5}; do
        xv="WL_ARGS_$wl"  # per-workload flags (WL_ARGS_c3f="--steps 20"; the last --steps wins)
        timeout -k 10 900 python bench.py --workload $wl --steps 5 --warmup 2 ${WL_ARGS:-} ${!xv:-} > gpurun_out/wl_${TAG}_$wl.json 2> gpurun_out/wl_${TAG}_$wl.err
        rc=$?; echo "== $wl"; python tools/bench_brief.py gpurun_out/wl_${TAG}_$wl.json; tail -2 gpurun_out/wl_${TAG}_$wl.err; [ $rc -eq 0 ] || exit $rc
      done ;;
  esac
done
