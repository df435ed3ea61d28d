#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5fs; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stream_native.py > $O/gpu_tests_stream.txt 2>&1 || { tail -30 $O/gpu_tests_stream.txt; exit 1; }
tail -1 $O/gpu_tests_stream.txt
bash tools/recipes/r5_c1bench.sh
for z in 0 1 2; do
  for a in "16 1 1" "16 64 8"; do
    ATLS_ZERO_COPY=$z timeout -k 10 60 tools/c1_loopback_native $a | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('zero_copy $z', d['conns'], d['reps'], d['threads'], d['verified'], d['gpu_MBps'], d['phase_ms'])" || exit 1
  done
done
