#!/bin/bash
# ChaCha step windows vs cache lines: RAW 1,536-B records with the input / output shifted by 64 B, so a
# 2-lane step's 128-B window (data blocks 2t-1, 2t) is line-aligned.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; O=gpurun_out/traffic3; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for v in "0 0" "64 64" "64 0" "0 64"; do
  set -- $v
  for pass in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    tag=raw_i$1_o$2_$(echo $pass | cut -c9-13)
    timeout -s KILL 90 rocprofv3 --pmc $pass -d $O/$tag -o run --output-format csv -- python3 tools/traffic_probe.py --config c3 --raw 1536 --out-align 1536 --in-align 1536 --in-shift $1 --out-shift $2 > $O/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -3 $O/$tag.log; exit 1; }
    echo "$tag ok"
  done
done
