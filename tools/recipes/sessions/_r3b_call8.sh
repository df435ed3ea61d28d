#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 tools/ubench/pcie_probe > gpurun_out/pcie_probe2.log 2>&1 || { echo "probe rc=$?"; cat gpurun_out/pcie_probe2.log; exit 1; }
grep -E "2d|both|chunk32" gpurun_out/pcie_probe2.log
bash tools/recipes/sessions/_ab_c3_traffic.sh 2>&1 | tee gpurun_out/ab_c3_carry.log
