#!/bin/bash
# The resident server's two modes on one build: the resident tests, then single-call floors, 3 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5rm; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_single_resident.py tests/test_gpu_single_call.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2 3; do
  for m in 1 2; do
    ATLS_SINGLE_RESIDENT=$m timeout -k 10 120 ./tools/single_call_floor > $O/floor_mode${m}_$r.json 2>&1 || { tail -5 $O/floor_mode${m}_$r.json; exit 1; }
    python3 -c "import json; d=json.load(open('$O/floor_mode${m}_$r.json')); print('round $r mode $m', {k: d[k] for k in ('chacha20poly1305_1537_seal_us','chacha20poly1305_1537_open_us','aes128gcm_1537_seal_us','aes128gcm_1537_open_us')})"
  done
done
