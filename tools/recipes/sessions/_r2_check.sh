#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/tests_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/tests_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/single_call_latency.py > gpurun_out/single_call_latency.json 2> gpurun_out/single_call_latency.err; echo lat rc=$?
cat gpurun_out/single_call_latency.json
