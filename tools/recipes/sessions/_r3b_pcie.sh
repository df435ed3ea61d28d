#!/bin/bash
# Round 3 (second session): PCIe probe (DMA vs kernel zero-copy, tools/ubench/pcie_probe.hip) beside the
# engine's host-memory C2 rate, then the wave-state PMC of the C3 ChaCha seal kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 180 tools/ubench/pcie_probe > gpurun_out/pcie_probe.log 2>&1 || { echo "probe rc=$?"; cat gpurun_out/pcie_probe.log; exit 1; }
cat gpurun_out/pcie_probe.log
timeout -k 10 300 python bench.py --pcie --no-cpu-baseline --no-open > gpurun_out/b_c2_pcie.log 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -1 gpurun_out/b_c2_pcie.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pcie_inclusive', d.get('pcie_inclusive_GiBps'), 'value', d['value'])"
bash tools/pmc_stall.sh c3_chacha20poly1305_64Ki_x_1.5KiB > gpurun_out/pmc_c3.log 2>&1 || { echo "pmc rc=$?"; tail gpurun_out/pmc_c3.log; exit 1; }
for p in a b; do python3 tools/pmc_summary.py $(ls gpurun_out/pmc_stall_$p/*/run_counter_collection.csv gpurun_out/pmc_stall_$p/run_counter_collection.csv 2>/dev/null | head -1) chacha_kernel 2; done
