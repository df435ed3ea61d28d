#!/bin/bash
# GPU tests named on the command line (default: all -m gpu), one process, per-test timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${@:-tests}" > gpurun_out/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/tests.log | tail -5; exit $rc
