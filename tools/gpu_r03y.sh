# C2 knob A/B: GPU allow-path prefilter, verify / finalize grid sizes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03y}
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --ingest-steps 0 > gpurun_out/bench_${T}_$n.json 2> gpurun_out/bench_${T}_$n.err
  local rc=$?
  python -c "import json;d=json.load(open('gpurun_out/bench_${T}_$n.json'));b=d['breakdown_ms'];print('$n',d['value'],d['ms_per_step'],b['ms_gpu_total'],b['ms_scan_kernel'],b['ms_nfa_kernel'],b['ms_finalize_kernel'],d['host_cpu']['process_cpu_ms_per_step'])"
  return $rc
}
run base TSG_X=0 && run noap TSG_GPU_ALLOW_PATH=0 && run v8k TSG_VERIFY_BLOCKS=8192 && run v2k TSG_VERIFY_BLOCKS=2048 && run f32k TSG_FINALIZE_BLOCKS=32768 && run base2 TSG_X=0
