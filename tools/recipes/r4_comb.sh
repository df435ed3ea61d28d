#!/bin/bash
# Round 4: the lane combine through a per-lane LDS table (ATLS_COMB_LDS, gcm_common.h gf_mul_comb_lds)
# against the register comb: GCM / ChaCha parity of the default build, the AES-GCM single-call phase
# clocks of both timing builds, then the same-box A/B of both variants on C5, C2 and C4 (tools/recipes/r4_ab.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gcm_groups.py tests/test_gpu_single_call.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4/comb_parity.txt 2>&1 || { tail -30 gpurun_out/r4/comb_parity.txt; exit 1; }
tail -2 gpurun_out/r4/comb_parity.txt
for v in ttstamps tt2; do
  ATLS_LIB=$PWD/anothertls_amd/variants/libatls_$v.so timeout -k 10 180 python3 tools/tt_stamps_single.py > gpurun_out/r4/comb_stamps_$v.json 2>&1 || { cat gpurun_out/r4/comb_stamps_$v.json; exit 1; }
  cat gpurun_out/r4/comb_stamps_$v.json
done
VARIANTS="${VARIANTS:-base comb1 comb2}" CONFIGS="${CONFIGS:-c5_mixed_256Ki_x_64B-16KiB c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB}" ROUNDS=3 bash tools/recipes/r4_ab.sh ${TAG:-comb}
