#!/bin/bash
# Same-box A/B: kernel time of each anothertls_amd/variants/libatls_*.so (interleaved, 2 rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cfg=${1:-c2_aes128gcm_64Ki_x_16KiB}
for round in 1 2; do
  for lib in anothertls_amd/variants/libatls_*.so; do
    r=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --steps 10 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])") || exit $?
    echo "round $round $(basename $lib): $r"
  done
done
