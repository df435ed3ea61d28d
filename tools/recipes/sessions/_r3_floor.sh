#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; O=gpurun_out/floor; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 120 ./tools/single_call_floor > $O/floor.json 2> $O/floor.err || { echo "floor rc=$?"; cat $O/floor.err; exit 1; }
cat $O/floor.json
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- ./tools/single_call_floor > $O/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo done
