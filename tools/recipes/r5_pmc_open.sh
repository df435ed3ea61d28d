#!/bin/bash
# Seal against open kernel of C2 (gcm_kernel<false/true, 12, 10>): wave-state and pipe PMC passes, each its own run
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5po; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
have() { for c in "$@"; do grep -qw "$c" $O/counters.txt && printf '%s ' "$c"; done; }
A=$(have SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES)
B=$(have SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INST_CYCLES_SALU)
echo "pass a: $A"; echo "pass b: $B"
CMD="python3 bench.py --config c2_aes128gcm_64Ki_x_16KiB --steps 5 --warmup 2 --no-cpu-baseline --no-configs --sustain-s 0 --load-settle-ms 100"
timeout -s KILL 120 rocprofv3 --pmc $A GRBM_GUI_ACTIVE -d $O/a -o run --output-format csv -- $CMD > $O/a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $B GRBM_GUI_ACTIVE -d $O/b -o run --output-format csv -- $CMD > $O/b.log 2>&1 || exit $?
for p in a b; do
  f=$(ls $O/$p/*/run_counter_collection.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls $O/$p/run_counter_collection.csv)
  python3 tools/pmc_summary.py $f gcm_kernel 2 > $O/summary_$p.json
  cat $O/summary_$p.json
done
