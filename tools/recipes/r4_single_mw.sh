#!/bin/bash
# Round 4: the single-call AES-GCM record on four waves (gcm_record LN = 256; gcm_single / gcm_single_ptr):
# every GPU test, then the single-call floors and latencies and the AES-GCM single-call phase clocks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/mw_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r4/mw_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r4/mw_gpu_tests.txt
timeout -k 10 120 ./tools/single_call_floor > gpurun_out/r4/mw_single_call_floor.json 2>&1 || { cat gpurun_out/r4/mw_single_call_floor.json; exit 1; }
timeout -k 10 300 python3 tools/single_call_latency.py > gpurun_out/r4/mw_single_call_latency.json 2>&1 || { cat gpurun_out/r4/mw_single_call_latency.json; exit 1; }
ATLS_LIB=$PWD/anothertls_amd/variants/libatls_ttstamps.so timeout -k 10 180 python3 tools/tt_stamps_single.py > gpurun_out/r4/mw_stamps.json 2>&1 || { cat gpurun_out/r4/mw_stamps.json; exit 1; }
cat gpurun_out/r4/mw_single_call_floor.json gpurun_out/r4/mw_single_call_latency.json gpurun_out/r4/mw_stamps.json
