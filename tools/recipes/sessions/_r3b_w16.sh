#!/bin/bash
# Timing-only: the GCM kernel at 16 waves per CU (one GHASH table per workgroup, wrong tags on purpose:
# ATLS_DBG_SHARED_GHASH) against 12 waves with and without the shared table, C2 and C4, 3 rounds; then
# the LDS wave-state PMC of the 12- and 16-wave shared builds on C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out/w16
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
V=anothertls_amd/variants
for round in 1 2 3; do
  for spec in "a_cur 12" "b_shared 12" "b_shared 16"; do
    set -- $spec
    for c in c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB; do
      r=$(ATLS_GCM_WAVES=$2 ATLS_LIB=$PWD/$V/libatls_$1.so timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --no-open 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'seal', d['roofline']['kernel_ms'])") || exit 1
      echo "round $round $1 waves=$2 ${c%%_*}: $r"
    done
  done
done
CMD="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-open"
for spec in "b_shared 12" "b_shared 16"; do
  set -- $spec
  ATLS_GCM_WAVES=$2 ATLS_LIB=$PWD/$V/libatls_$1.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/w16/pmc_$1_$2 -o run --output-format csv -- $CMD > gpurun_out/w16/pmc_$1_$2.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/w16/pmc_$1_$2/run_counter_collection.csv gcm_kernel 2 | python3 -c "
import json,sys; d=json.load(sys.stdin)
for k,v in d.items(): print('$1 $2', k.split('(')[0], {x:v[x] for x in v if x!='avg'})"
done
