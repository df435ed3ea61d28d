#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ATLS_LIB=$PWD/anothertls_amd/variants/libatls_b_pre3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chacha_widths.py tests/test_gpu_configs.py::test_c3_full_batch_device_resident_vs_openssl_and_oracle tests/test_wire_mode.py -p no:cacheprovider > gpurun_out/par_pre3.log 2>&1 || { echo "pre3 parity FAIL"; tail -20 gpurun_out/par_pre3.log; exit 1; }
echo "pre3 parity: $(tail -1 gpurun_out/par_pre3.log)"
bash tools/recipes/sessions/_ab_c3_time.sh
