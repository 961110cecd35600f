#!/bin/bash
# Host C++ under sanitizers: ASan+UBSan and TSan builds of the
# host library (oracle/build/libtsg_host.so's sources: the product's host C++ --
# rule compiler, Go-regexp engine, exact tail, analyzer/tar walker, C-ABI -- plus
# the oracle hooks), driven by the CPU tests that exercise them: the exact tail
# (whole-file windows), the reference scan's file fan-out and concurrent scans
# on one scanner (tests/test_host_concurrency.py), the collector / tar walk /
# Required (tests/test_analyzer.py) and the allow-path pass.  The gfx950 device
# code (engine.hip) is linked unsanitized: no GPU runs here.
# Usage: bash tools/sanitize.sh [asan|tsan|all]   (logs -> profiles/sanitize_*.log)
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd)
MODE=${1:-all}
python -c "import __graft_entry__ as g; g.build()" || exit 1
COMMON="-O1 -g -march=x86-64-v3 -fPIC -std=c++17 -fno-omit-frame-pointer -I trivy_amd/csrc -I include -I oracle/native -D__HIP_PLATFORM_AMD__ -I /opt/rocm/include"
TESTS="tests/test_host_concurrency.py tests/test_host_tail.py tests/test_analyzer.py tests/test_allow_path.py tests/test_rules_data.py tests/test_fs_walk.py"
build() {  # $1 = name, $2 = sanitizer flags
  local out=oracle/build/san_$1
  mkdir -p $out
  local objs=""
  for src in trivy_amd/csrc/*.cpp oracle/native/*.cpp; do
    local o=$out/$(basename ${src%.cpp}).o
    g++ $COMMON $2 -c $src -o $o || return 1
    objs="$objs $o"
  done
  g++ -shared $2 -o $out/libtsg_host.so $objs trivy_amd/_obj/*.hip.o -L/opt/rocm/lib -lamdhip64 -lpthread \
    -Wl,-rpath,/opt/rocm/lib || return 1
  echo $out/libtsg_host.so
}
rc=0
if [ "$MODE" = asan ] || [ "$MODE" = all ]; then
  lib=$(build asan "-fsanitize=address,undefined -fno-sanitize-recover=undefined") || exit 1
  LD_PRELOAD=$(g++ -print-file-name=libasan.so):$(g++ -print-file-name=libubsan.so) \
  ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  TSG_HOSTLIB=$ROOT/$lib python -m pytest $TESTS -q -m "not gpu" -p no:cacheprovider > profiles/sanitize_${SAN_TAG:-r06}_asan_ubsan.log 2>&1
  r=$?; tail -3 profiles/sanitize_${SAN_TAG:-r06}_asan_ubsan.log; [ $r -eq 0 ] || rc=$r
fi
if [ "$MODE" = tsan ] || [ "$MODE" = all ]; then
  lib=$(build tsan "-fsanitize=thread") || exit 1
  # The TSan runtime must be preloaded into the interpreter: dlopen of a TSan-built library
  # otherwise fails with "cannot allocate memory in static TLS block" (round 3's failure: a
  # comment line inside this command's continuation had dropped the preload).  The
  # pool-budget test spawns interpreters that inherit the preload and stall in it: not a
  # race test, deselected.
  LD_PRELOAD=$(readlink -f $(g++ -print-file-name=libtsan.so)) \
  TSAN_OPTIONS=halt_on_error=1:report_signal_unsafe=0:second_deadlock_stack=1 \
  TSG_HOSTLIB=$ROOT/$lib python -m pytest ${TSAN_TESTS:-tests/test_host_concurrency.py tests/test_host_tail.py tests/test_analyzer.py} \
    -q -m "not gpu" -k "not pool_budget and not pool_spare" -p no:cacheprovider > profiles/sanitize_${SAN_TAG:-r06}_tsan.log 2>&1
  r=$?; tail -3 profiles/sanitize_${SAN_TAG:-r06}_tsan.log; [ $r -eq 0 ] || rc=$r
fi
exit $rc
