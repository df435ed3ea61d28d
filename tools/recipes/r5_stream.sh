#!/bin/bash
# Round 5: the multi-threaded socket path (tests, C1 at scale) and the full GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5st; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream_native.py -x -v --timeout 200 --timeout-method thread > $O/gpu_tests_stream.txt 2>&1 || { tail -40 $O/gpu_tests_stream.txt; exit 1; }
tail -1 $O/gpu_tests_stream.txt
for a in "8 64 1" "8 64 4" "8 64 8" "8 64 16" "2 256 8" "2 256 16"; do timeout -k 10 120 tools/c1_loopback_native $a || exit 1; done > $O/c1_scale.log 2>&1
cat $O/c1_scale.log
timeout -k 10 400 python -u bench.py --config c1_server_https_loopback_1MiB --steps 8 > $O/bench_c1.json 2> $O/bench_c1.err || { tail -20 $O/bench_c1.err; exit 1; }
cat $O/bench_c1.json
