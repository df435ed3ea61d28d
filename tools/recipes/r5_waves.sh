#!/bin/bash
# AES-GCM waves per workgroup (ATLS_GCM_WAVES: 12 = default, 8) on C2 / C4 / C5, 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for r in 1 2; do
  for w in 12 8; do
    for cfg in c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB c5_mixed_256Ki_x_64B-16KiB; do
      ATLS_GCM_WAVES=$w timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-configs --sustain-s 0 --steps 10 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('round $r waves $w $cfg', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['open']['kernel_ms'], d['open']['plaintext_and_status_ok'])" || exit 1
    done
  done
done
