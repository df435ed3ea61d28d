#!/bin/bash
# Round 4: the 4-wave AES-GCM single call building only the tables a record uses -- single-call and parity
# tests, floors / latencies, phase clocks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_gpu_single_call.py tests/test_gpu_parity.py tests/test_abi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/tab_tests.txt 2>&1 || { tail -40 gpurun_out/r4/tab_tests.txt; exit 1; }
tail -1 gpurun_out/r4/tab_tests.txt
timeout -k 10 120 ./tools/single_call_floor > gpurun_out/r4/tab_single_call_floor.json 2>&1 || { cat gpurun_out/r4/tab_single_call_floor.json; exit 1; }
ATLS_LIB=$PWD/anothertls_amd/variants/libatls_ttstamps.so timeout -k 10 180 python3 tools/tt_stamps_single.py > gpurun_out/r4/tab_stamps.json 2>&1 || { cat gpurun_out/r4/tab_stamps.json; exit 1; }
cat gpurun_out/r4/tab_single_call_floor.json gpurun_out/r4/tab_stamps.json
