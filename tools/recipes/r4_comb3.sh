#!/bin/bash
# Round 4: single-call first step + LDS lane combine follow-up: single-call tests (incl. the first-step
# boundary), AES-GCM single-call phase clocks, then base / comb1 / combu1 (rolled loop) / comb256off
# (AES-256 keeps the register comb) on C4, C5 and C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_single_call.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4/comb3_single_tests.txt 2>&1 || { tail -30 gpurun_out/r4/comb3_single_tests.txt; exit 1; }
tail -2 gpurun_out/r4/comb3_single_tests.txt
ATLS_LIB=$PWD/anothertls_amd/variants/libatls_ttstamps.so timeout -k 10 180 python3 tools/tt_stamps_single.py > gpurun_out/r4/comb3_stamps.json 2>&1 || { cat gpurun_out/r4/comb3_stamps.json; exit 1; }
cat gpurun_out/r4/comb3_stamps.json
timeout -k 10 200 python3 tools/single_call_latency.py > gpurun_out/r4/comb3_single_latency.json 2>&1 || { cat gpurun_out/r4/comb3_single_latency.json; exit 1; }
cat gpurun_out/r4/comb3_single_latency.json
VARIANTS="base comb1 combu1 comb256off" CONFIGS="c4_aes256gcm_1Mi_x_16KiB c5_mixed_256Ki_x_64B-16KiB c2_aes128gcm_64Ki_x_16KiB" ROUNDS=3 bash tools/recipes/r4_ab.sh comb3
