#!/bin/bash
# Round 6: (1) the product (C5's mixed-batch seal capped at 128 VGPRs) against ATLS_GCM_FAST_FIRST=1 on C2 with a key per
# record, C5 and C2, parity first; (2) C3's per-record share priced part by part with ATLS_CHACHA_DBG timing builds
# (wrong results on purpose: no parity): 1 data keystream, 2 MAC, 8 r-power scan, 16 lane-combine products,
# 32 tag finish, 64 power products, 120 = 8|16|32|64. Outputs gpurun_out/r6/ab_{keyrec,c3parts}.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
PARITY_TESTS="tests/test_gpu_plan.py tests/test_gpu_configs.py tests/test_gpu_gcm_groups.py tests/test_gpu_parity.py" \
VARIANTS="base fastfirst" CONFIGS="c2_aes128gcm_64Ki_x_16KiB:0:65536 c5_mixed_256Ki_x_64B-16KiB:262144 c5_mixed_256Ki_x_64B-16KiB c2_aes128gcm_64Ki_x_16KiB" \
  ROUNDS=3 bash tools/recipes/r6_ab.sh keyrec || exit 1
PARITY=0 VARIANTS="base dbg1 dbg2 dbg8 dbg16 dbg32 dbg64 dbg120" CONFIGS="c3_chacha20poly1305_64Ki_x_1.5KiB" ROUNDS=3 \
  bash tools/recipes/r6_ab.sh c3parts
