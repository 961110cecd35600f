# A/B of engine knobs on bench.py: one bench per setting.  A setting is
# "ENV=V ... [:: bench args]"; settings are separated by ';'.
# Usage: gpurun -- 'TAG=r02k AB="X=0;TSG_DIAG_CONFIRM=32;X=0 :: --workload c3" bash tools/gpu_ab.sh'
set -o pipefail
TAG=${TAG:-ab}
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${AB:-X=0}"
i=0
for s in "${SETS[@]}"; do
  e=${s%%::*}; a=""; [[ "$s" == *::* ]] && a=${s#*::}
  env $e timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} $a > gpurun_out/ab_${TAG}_$i.json 2> gpurun_out/ab_${TAG}_$i.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_${TAG}_$i.err; exit $rc; }
  echo "== $s"; python tools/bench_brief.py gpurun_out/ab_${TAG}_$i.json
  i=$((i+1))
done
