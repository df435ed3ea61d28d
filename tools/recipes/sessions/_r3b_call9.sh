#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_host_pipeline.py -p no:cacheprovider > gpurun_out/t9.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t9.log; exit 1; }
tail -1 gpurun_out/t9.log
for mb in 32 64; do
  ATLS_CHUNK_MB=$mb timeout -k 10 300 python bench.py --pcie --no-cpu-baseline --no-open --steps 5 > gpurun_out/b_pcie_$mb.log 2>&1 || { echo "bench rc=$?"; tail gpurun_out/b_pcie_$mb.log; exit 1; }
  tail -1 gpurun_out/b_pcie_$mb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunk $mb: staged', d.get('pcie_inclusive_GiBps'), 'zc', d.get('pcie_zero_copy_GiBps'), d.get('pcie_zero_copy_equal'), 'zc_out', d.get('pcie_zero_copy_out_GiBps'), d.get('pcie_zero_copy_out_equal'))"
done
timeout -k 10 120 tools/ubench/pcie_probe 2>&1 | grep -E "dma_both|dma_chunk32|d2h_2d" 
