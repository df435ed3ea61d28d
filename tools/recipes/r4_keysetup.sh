#!/bin/bash
# Round 4: the one-wave-per-key key-setup kernel -- every GPU test, the key-install timings (with a
# rocprof kernel trace) and the single-call latencies with a fresh key per call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/gpu_tests_keysetup.txt 2>&1 || { tail -30 gpurun_out/r4/gpu_tests_keysetup.txt; exit 1; }
tail -3 gpurun_out/r4/gpu_tests_keysetup.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_keysetup -o run --output-format csv -- python3 tools/key_setup_bench.py > gpurun_out/r4/key_setup_bench.json 2> gpurun_out/r4/key_setup_bench.err || exit 1
cat gpurun_out/r4/key_setup_bench.json
timeout -k 10 300 python3 tools/single_call_latency.py > gpurun_out/r4/single_call_latency.json 2>&1 || exit 1
cat gpurun_out/r4/single_call_latency.json
