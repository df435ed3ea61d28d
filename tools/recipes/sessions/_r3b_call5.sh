#!/bin/bash
# Round 3 (second session): host-memory batches (staged three-stream pipeline, zero copy) and ChaCha
# defaults (SOP seals, 2-wave opens): their tests, then C2 --pcie and C3 / C5 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_host_pipeline.py tests/test_gpu_chacha_widths.py tests/test_gpu_configs.py tests/test_wire_mode.py tests/test_gpu_parity.py -p no:cacheprovider > gpurun_out/t5.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error|error" gpurun_out/t5.log | head -20; tail -30 gpurun_out/t5.log; exit 1; }
tail -1 gpurun_out/t5.log
timeout -k 10 300 python bench.py --pcie --no-cpu-baseline --no-open > gpurun_out/b_c2_pcie.log 2>&1 || { echo "bench rc=$?"; tail gpurun_out/b_c2_pcie.log; exit 1; }
tail -1 gpurun_out/b_c2_pcie.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pcie staged', d.get('pcie_inclusive_GiBps'), 'zero copy', d.get('pcie_zero_copy_GiBps'), d.get('pcie_zero_copy_equal'), 'value', d['value'])"
for c in c3_chacha20poly1305_64Ki_x_1.5KiB c5_mixed_256Ki_x_64B-16KiB; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/b_$c.log 2>&1 || { echo "$c rc=$?"; exit 1; }
  tail -1 gpurun_out/b_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], 'open', d['open'])"
done
