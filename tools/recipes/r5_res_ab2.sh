#!/bin/bash
# The both-suites server (ATLS_SINGLE_RESIDENT=2) built three ways: base (217 VGPRs), minw4 (capped at 128),
# nr10 (the AES-GCM path for 10 rounds only); floors of both suites, 3 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5rab2; mkdir -p $O
for r in 1 2 3; do
  for v in ${VARS:-base minw4 nr10}; do
    LD_LIBRARY_PATH=$PWD/anothertls_amd/variants/d_$v ATLS_SINGLE_RESIDENT=2 timeout -k 10 120 ./tools/single_call_floor > $O/floor_${v}_$r.json 2>&1 || { tail -5 $O/floor_${v}_$r.json; exit 1; }
    python3 -c "import json; d=json.load(open('$O/floor_${v}_$r.json')); print('round $r $v', {k: d[k] for k in ('chacha20poly1305_1537_seal_us','chacha20poly1305_1537_open_us','aes128gcm_1537_seal_us','aes128gcm_1537_open_us')})"
  done
done
