#!/bin/bash
# Round 5 A/B: general steps with EXEC-masked AES / GHASH on the lanes past the record (ATLS_GEN_MASK=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
PARITY=1 VARIANTS="base mask" CONFIGS="c5_mixed_256Ki_x_64B-16KiB c4_aes256gcm_1Mi_x_16KiB" ROUNDS=3 timeout -k 10 1200 bash tools/recipes/r5_ab.sh genmask || exit 1
PARITY=0 VARIANTS="base mask" CONFIGS="c2_aes128gcm_64Ki_x_16KiB" BENCH_ARGS="--key-slots 65536" ROUNDS=3 timeout -k 10 600 bash tools/recipes/r5_ab.sh genmask_keyrec || exit 1
