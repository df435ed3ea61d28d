#!/bin/bash
# Timing-only A/B of anothertls_amd/variants/libatls_*.so on C3 (no parity: ATLS_CHACHA_DBG builds compute
# wrong results on purpose), 3 interleaved rounds of the seal kernel time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2 3; do
  for lib in anothertls_amd/variants/libatls_*.so; do
    n=$(basename $lib .so)
    r=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --no-cpu-baseline --no-open 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'seal', d['roofline']['kernel_ms'])") || exit 1
    echo "round $round $n: C3 $r"
  done
done
