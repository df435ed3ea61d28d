#!/bin/bash
# Round-3 check on one box: the GPU test suite, the C2 bench line (seal + open), and the single-call
# latency at three zero-copy thresholds. Stops at the first step that faults, aborts or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  echo "[$(date +%T)] $name" >> gpurun_out/r3_steps.log
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> gpurun_out/r3_steps.log
  echo "$name rc=$rc: $(tail -1 "gpurun_out/$name.log" | cut -c1-600)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    tests) step tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider ;;
    bench) step bench 600 python bench.py ;;
    lat) for zc in 4096 0 1000000; do ATLS_SINGLE_ZC_MAX=$zc step lat_zc$zc 300 python tools/single_call_latency.py; done ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
