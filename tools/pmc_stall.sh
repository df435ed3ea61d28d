#!/bin/bash
# Where the AES-GCM record kernel's waves spend their cycles (C2, product library): one SQ pass
# with the wave-state counters (MI355X_MICROARCH.md "rocprofv3 PMC slots": WAIT_ANY = parked at
# s_waitcnt, WAIT_INST_ANY = issue stall, ACTIVE_INST_ANY = issuing; together ~ WAVE_CYCLES) and
# one with the per-pipe activity. Counters the tool does not list on this box are left out.
# Outputs: gpurun_out/pmc_stall_{a,b}/ and gpurun_out/counters.txt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
have() { for c in "$@"; do grep -qw "$c" gpurun_out/counters.txt && printf '%s ' "$c"; done; }
A=$(have SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES)
B=$(have SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM)
echo "pass a: $A"; echo "pass b: $B"
CMD="python3 bench.py --config ${1:-c2_aes128gcm_64Ki_x_16KiB} --steps 5 --warmup 2 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc $A GRBM_GUI_ACTIVE -d gpurun_out/pmc_stall_a -o run --output-format csv -- $CMD > gpurun_out/pmc_stall_a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $B GRBM_GUI_ACTIVE -d gpurun_out/pmc_stall_b -o run --output-format csv -- $CMD > gpurun_out/pmc_stall_b.log 2>&1 || exit $?
echo done
