#!/bin/bash
# C3-shaped batches past two waves per SIMD (2x and 4x the records): the 3-wave kernel (default) against
# the 2-wave kernel forced (ATLS_CHACHA_W2=2), seal and open, 3 interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2 3; do
  for recs in 131072 262144; do
    for w2 in 1 2; do
      r=$(ATLS_CHACHA_W2=$w2 timeout -k 10 120 python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --records $recs --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'seal', d['roofline']['kernel_ms'], 'open', d['open']['kernel_ms'], d['open']['plaintext_and_status_ok'])") || exit 1
      echo "round $round records=$recs w2=$w2: $r"
    done
  done
done
