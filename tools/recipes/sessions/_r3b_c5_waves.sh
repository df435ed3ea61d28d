#!/bin/bash
# C5 (AES-GCM kernel beside the planned ChaCha20-Poly1305 kernel): GCM waves per workgroup x ChaCha
# workgroups per CU, product library, 3 interleaved rounds (env knobs only; no rebuild).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2 3; do
  for spec in "12 8" "8 8" "8 16" "12 16"; do
    set -- $spec
    r=$(ATLS_GCM_WAVES=$1 ATLS_CHACHA_WGS=$2 timeout -k 10 120 python bench.py --config c5_mixed_256Ki_x_64B-16KiB --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'seal', d['roofline']['kernel_ms'], 'open', d['open']['kernel_ms'])") || exit 1
    echo "round $round gcm_waves=$1 chacha_wgs=$2: C5 $r"
  done
done
