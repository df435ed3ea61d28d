#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5sc4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_single_resident.py tests/test_gpu_single_call.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_single.txt 2>&1 || { tail -40 $O/gpu_tests_single.txt; exit 1; }
tail -1 $O/gpu_tests_single.txt
for m in 0 1 2; do
  ATLS_SINGLE_RESIDENT=$m timeout -k 10 200 ./tools/single_call_floor > $O/single_call_floor_mode$m.json 2>&1 || { tail -5 $O/single_call_floor_mode$m.json; exit 1; }
  echo "mode $m: $(cat $O/single_call_floor_mode$m.json)"
done
