#!/bin/bash
# Round 4: C4 at its stated size (1 Mi x 16 KiB on one GPU, one engine and the RCCL-self 8-part layout),
# the single-call tests (argument-block kernels), the default bench line (C2 + the C3 / C4-shard /
# C5-shard configs), key-install timings and single-call latencies.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_single_call.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4/gpu_tests_single.txt 2>&1 || { tail -40 gpurun_out/r4/gpu_tests_single.txt; exit 1; }
tail -2 gpurun_out/r4/gpu_tests_single.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_c4_full.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r4/gpu_tests_c4_full.txt 2>&1 || { tail -40 gpurun_out/r4/gpu_tests_c4_full.txt; exit 1; }
tail -4 gpurun_out/r4/gpu_tests_c4_full.txt
s=$(python3 -c "import time; print(time.time())")
timeout -k 10 300 python -u bench.py > gpurun_out/r4/bench_default.json 2> gpurun_out/r4/bench_default.err || { tail -20 gpurun_out/r4/bench_default.err; exit 1; }
e=$(python3 -c "import time; print(time.time())")
python3 -c "print('bench wall: %.1f s' % ($e - $s))"
cat gpurun_out/r4/bench_default.json
timeout -k 10 300 python3 tools/key_setup_bench.py > gpurun_out/r4/key_setup_bench2.json 2>&1 || exit 1
cat gpurun_out/r4/key_setup_bench2.json
timeout -k 10 300 python3 tools/single_call_latency.py > gpurun_out/r4/single_call_latency2.json 2>&1 || exit 1
cat gpurun_out/r4/single_call_latency2.json
