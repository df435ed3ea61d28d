#!/bin/bash
# Round measurements: default bench (CPU baseline + PCIe-inclusive), C3, C4 (per-GPU share), C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --pcie > gpurun_out/m_c2.log 2>&1 || exit $?
tail -1 gpurun_out/m_c2.log
timeout -k 10 200 python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --no-cpu-baseline > gpurun_out/m_c3.log 2>&1 || exit $?
tail -1 gpurun_out/m_c3.log
timeout -k 10 300 python bench.py --config c4_aes256gcm_1Mi_x_16KiB --no-cpu-baseline --steps 5 > gpurun_out/m_c4.log 2>&1 || exit $?
tail -1 gpurun_out/m_c4.log
timeout -k 10 300 python bench.py --config c5_mixed_256Ki_x_64B-16KiB --no-cpu-baseline --steps 5 > gpurun_out/m_c5.log 2>&1 || exit $?
tail -1 gpurun_out/m_c5.log
