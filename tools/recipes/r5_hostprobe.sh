#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5hp; mkdir -p $O
timeout -k 10 300 python -u tools/host_batch_probe.py > $O/host_batch_probe.log 2>&1 || { tail -20 $O/host_batch_probe.log; exit 1; }
cat $O/host_batch_probe.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream_native.py tests/test_gpu_host_pipeline.py tests/test_wire_mode.py -x -v --timeout 200 --timeout-method thread > $O/gpu_tests_stream.txt 2>&1 || { tail -40 $O/gpu_tests_stream.txt; exit 1; }
tail -1 $O/gpu_tests_stream.txt
for a in "8 64 1" "8 64 4" "8 64 8" "8 64 16" "2 256 8" "2 256 16"; do ATLS_SB_PROFILE=1 timeout -k 10 120 tools/c1_loopback_native $a || exit 1; done > $O/c1_scale.log 2>&1
cat $O/c1_scale.log
PARITY=0 VARIANTS="base skip1 skip4 skip2 skip16 skip32" CONFIGS="c2_aes128gcm_64Ki_x_16KiB" BENCH_ARGS="--key-slots 65536" ROUNDS=3 timeout -k 10 900 bash tools/recipes/r5_ab.sh keyrec_parts || exit 1
timeout -k 10 200 ./tools/single_call_floor > gpurun_out/r5hp/single_call_floor.json 2>&1 || { tail -5 gpurun_out/r5hp/single_call_floor.json; exit 1; }
cat gpurun_out/r5hp/single_call_floor.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_single_call.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5hp/gpu_tests_single.txt 2>&1 || { tail -40 gpurun_out/r5hp/gpu_tests_single.txt; exit 1; }
tail -1 gpurun_out/r5hp/gpu_tests_single.txt
