#!/bin/bash
# Same-box A/B of key-grouped direct AES-GCM batches: ATLS_GCM_GROUP_MIN=0 (off) vs default (on).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2 3; do
  for g in 0 2048; do
    for cfg in c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB; do
      r=$(ATLS_GCM_GROUP_MIN=$g timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])") || exit 1
      echo "round $round group_min=$g $cfg: $r"
    done
  done
done
