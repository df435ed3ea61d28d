#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/recipes/sessions/_ab_c3.sh 2>&1 | tee gpurun_out/ab_c3.log; [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_host_pipeline.py tests/test_gpu_chacha_widths.py tests/test_wire_mode.py -p no:cacheprovider > gpurun_out/t_host.log 2>&1 || { echo "host tests rc=$?"; tail -30 gpurun_out/t_host.log; exit 1; }
tail -1 gpurun_out/t_host.log
timeout -k 10 300 python bench.py --pcie --no-cpu-baseline --no-open > gpurun_out/b_c2_pcie.log 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -1 gpurun_out/b_c2_pcie.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pcie_inclusive', d.get('pcie_inclusive_GiBps'), 'value', d['value'])"
for mb in 8 32; do ATLS_CHUNK_MB=$mb timeout -k 10 300 python bench.py --pcie --no-cpu-baseline --no-open --steps 5 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunk $mb MiB pcie_inclusive', d.get('pcie_inclusive_GiBps'))" || exit 1; done
