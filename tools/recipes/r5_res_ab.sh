#!/bin/bash
# Resident server with and without the AES-GCM path (ATLS_RESIDENT_GCM=0): single-call floors, 3 rounds,
# variants in anothertls_amd/variants/d_<name>/libatls.so (the tool's RUNPATH gives way to LD_LIBRARY_PATH)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5rab; mkdir -p $O
for r in 1 2 3; do
  for v in ${VARS:-base nogcm}; do
    LD_LIBRARY_PATH=$PWD/anothertls_amd/variants/d_$v ATLS_SINGLE_RESIDENT=1 timeout -k 10 120 ./tools/single_call_floor > $O/floor_${v}_$r.json 2>&1 || { tail -5 $O/floor_${v}_$r.json; exit 1; }
    python3 -c "import json; d=json.load(open('$O/floor_${v}_$r.json')); print('round $r $v', {k: d[k] for k in ('chacha20poly1305_1537_seal_us','chacha20poly1305_1537_open_us','aes128gcm_1537_seal_us','aes128gcm_1537_open_us','resident_wave_doorbell_1552B_us')})"
  done
done
