#!/bin/bash
# Round 4: phase clocks of the one-record-per-wave AES-GCM path in batches (tools/tt_stamps.py, -DATLS_TT_STAMPS):
# C2 with a key per record (no lane groups), C5's AES-GCM records, C2 as configured.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
o=gpurun_out/r4/tt_batch.log
: > $o
timeout -k 10 200 python3 tools/tt_stamps.py c2_aes128gcm_64Ki_x_16KiB 65536 >> $o 2>&1 || { cat $o; exit 1; }
timeout -k 10 200 python3 tools/tt_stamps.py c5_mixed_256Ki_x_64B-16KiB >> $o 2>&1 || { cat $o; exit 1; }
timeout -k 10 200 python3 tools/tt_stamps.py c2_aes128gcm_64Ki_x_16KiB >> $o 2>&1 || { cat $o; exit 1; }
cat $o
