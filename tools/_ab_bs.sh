#!/bin/bash
# A/B of the bitsliced-step share (ATLS_GCM_BS) on one box: parity first, then C2/C4 benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ATLS_GCM_BS=16 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_parity.py > gpurun_out/bs_parity.log 2>&1 || { echo parity-fail; tail -30 gpurun_out/bs_parity.log; exit 1; }
tail -2 gpurun_out/bs_parity.log
for cfg in c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB; do
for bs in 0 8 16 0 8 16; do
  ATLS_GCM_BS=$bs timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --steps 20 > gpurun_out/ab_${cfg}_${bs}.json 2>gpurun_out/ab_err.log || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_${cfg}_${bs}.json').read().strip().splitlines()[-1]); print('$cfg', 'BS=$bs', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done; done
