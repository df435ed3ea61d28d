#!/bin/bash
# Same-box A/B of AES-GCM waves per workgroup 12 / 11 / 10 on C2 and C4 (library variant w), 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0 ATLS_LIB=$PWD/anothertls_amd/variants/libatls_w.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gcm_groups.py -p no:cacheprovider > gpurun_out/ab/wpar.log 2>&1 || { echo "parity rc=$?"; tail -5 gpurun_out/ab/wpar.log; exit 1; }
echo "parity (12 waves): $(tail -1 gpurun_out/ab/wpar.log)"
ATLS_GCM_WAVES=11 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gcm_groups.py tests/test_gpu_configs.py -p no:cacheprovider > gpurun_out/ab/wpar11.log 2>&1 || { echo "parity11 rc=$?"; tail -5 gpurun_out/ab/wpar11.log; exit 1; }
echo "parity (11 waves): $(tail -1 gpurun_out/ab/wpar11.log)"
for round in 1 2 3; do
  for w in 12 11 10; do
    for cfg in c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB; do
      ATLS_GCM_WAVES=$w timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/ab/w.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/ab/w.log; exit 1; }
      echo "round $round waves $w $cfg: $(tail -1 gpurun_out/ab/w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['open']['kernel_ms'])")"
    done
  done
done
