#!/bin/bash
# Kernel time vs record count at a fixed record length (C2's 16 KiB, and 1 KiB): intercept = per-launch cost.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in c2_aes128gcm_64Ki_x_16KiB; do
for n in 8192 16384 32768 49152 65536 98304 131072; do
  r=$(timeout -k 10 120 python bench.py --config $cfg --records $n --no-cpu-baseline --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])") || exit 1
  echo "$cfg records=$n: $r"
done; done
