#!/bin/bash
# Round 5: atls_clock_probe against the kernel's own s_memtime / s_memrealtime stamps (diagnostic build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5clk2; mkdir -p $O
ATLS_LIB=anothertls_amd/variants/libatls_clk.so timeout -k 10 300 python -u tools/clock_check.py --seconds 2 > $O/clock_check.json 2> $O/clock_check.err || { tail -30 $O/clock_check.err; exit 1; }
cat $O/clock_check.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_single_call.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_single.txt 2>&1 || { tail -30 $O/gpu_tests_single.txt; exit 1; }
tail -1 $O/gpu_tests_single.txt
