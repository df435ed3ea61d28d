#!/bin/bash
# Single-call latency floor (C ABI), C5 kernel trace (lazy join) and a C5 per-kernel pipe PMC pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; O=gpurun_out/c5prof; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 120 ./tools/single_call_floor > $O/single_call_floor.json 2> $O/single_call_floor.err || { echo "floor rc=$?"; cat $O/single_call_floor.err; exit 1; }
cat $O/single_call_floor.json
CMD="python3 bench.py --config c5_mixed_256Ki_x_64B-16KiB --steps 10 --warmup 2 --no-cpu-baseline --no-open"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $CMD > $O/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
tail -1 $O/trace.log | cut -c1-300
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/pmc -o run --output-format csv -- $CMD > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
echo done
