#!/bin/bash
# Round 4: both single-call ciphers on four waves -- every GPU test, then the single-call floors and latencies.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/mw2_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r4/mw2_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r4/mw2_gpu_tests.txt
timeout -k 10 120 ./tools/single_call_floor > gpurun_out/r4/mw2_single_call_floor.json 2>&1 || { cat gpurun_out/r4/mw2_single_call_floor.json; exit 1; }
timeout -k 10 300 python3 tools/single_call_latency.py > gpurun_out/r4/mw2_single_call_latency.json 2>&1 || { cat gpurun_out/r4/mw2_single_call_latency.json; exit 1; }
cat gpurun_out/r4/mw2_single_call_floor.json gpurun_out/r4/mw2_single_call_latency.json
