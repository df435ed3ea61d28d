#!/bin/bash
# C5's planned ChaCha20-Poly1305 kernel: lanes per record 16 (base) vs 32 (g32), 4 vs 3 waves per SIMD (w3);
# parity of each variant on the plan / config tests, then C5 shard and whole, 3 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5c5g; mkdir -p $O
for v in base g32 w3; do
  ATLS_LIB=$PWD/anothertls_amd/variants/libatls_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_configs.py tests/test_gpu_chacha_widths.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/parity_$v.txt 2>&1 || { echo "$v parity FAILED"; tail -20 $O/parity_$v.txt; continue; }
  echo "$v parity: $(tail -1 $O/parity_$v.txt)"
done
for r in 1 2 3; do
  for v in base g32 w3; do
    grep -q passed $O/parity_$v.txt || continue
    for rec in 32768 262144; do
      ATLS_LIB=$PWD/anothertls_amd/variants/libatls_$v.so timeout -k 10 200 python bench.py --config c5_mixed_256Ki_x_64B-16KiB --records $rec --no-cpu-baseline --no-configs --sustain-s 0 --steps 10 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('round $r $v $rec', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['open']['kernel_ms'], d['open']['plaintext_and_status_ok'])" || exit 1
    done
  done
done
