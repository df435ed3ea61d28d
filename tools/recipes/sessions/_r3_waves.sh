#!/bin/bash
# Same-box A/B of AES-GCM waves per workgroup (ATLS_GCM_WAVES 8 vs 12) on C2 / C4, interleaved, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2 3; do
  for w in 12 8; do
    for cfg in c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB; do
      ATLS_GCM_WAVES=$w timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/ab/w.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/ab/w.log; exit 1; }
      echo "round $round waves $w $cfg: $(tail -1 gpurun_out/ab/w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['open']['kernel_ms'])")"
    done
  done
done
