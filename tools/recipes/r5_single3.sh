#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5sc3; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_single_resident.py tests/test_gpu_single_call.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_single.txt 2>&1 || { tail -40 $O/gpu_tests_single.txt; exit 1; }
tail -1 $O/gpu_tests_single.txt
timeout -k 10 200 ./tools/single_call_floor > $O/single_call_floor.json 2>&1 || { tail -5 $O/single_call_floor.json; exit 1; }
cat $O/single_call_floor.json
ATLS_SINGLE_RESIDENT=1 timeout -k 10 200 ./tools/single_call_floor > $O/single_call_floor_resident.json 2>&1 || { tail -5 $O/single_call_floor_resident.json; exit 1; }
cat $O/single_call_floor_resident.json
