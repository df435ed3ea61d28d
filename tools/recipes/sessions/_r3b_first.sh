#!/bin/bash
# Round 3 (second session) first box: VALU op rates (valu2_ubench), the GPU suite and C2 / C3 bench lines on
# the restored tree, then the ChaCha A/B of anothertls_amd/variants (tools/recipes/sessions/_ab_chacha.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 tools/ubench/valu2_ubench > gpurun_out/valu2.log 2>&1 || { echo "ubench rc=$?"; exit 1; }
cat gpurun_out/valu2.log
bash tools/recipes/sessions/_run_tests.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/b_c2.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
tail -1 gpurun_out/b_c2.log | cut -c1-400
timeout -k 10 200 python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --no-cpu-baseline > gpurun_out/b_c3.log 2>&1 || { echo "c3 rc=$?"; exit 1; }
tail -1 gpurun_out/b_c3.log | cut -c1-400
bash tools/recipes/sessions/_ab_chacha.sh 2>&1 | tee gpurun_out/ab_chacha.log
