#!/bin/bash
# Read / write request counts of the ChaCha seal kernel with RAW 1,536-B records (every store a whole
# 16-B piece) at line-aligned and packed output strides, next to the TLS records of C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; O=gpurun_out/traffic2; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for v in "1536 128" "1536 16" "1536 1536"; do
  set -- $v
  for pass in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    tag=raw$1_o$2_$(echo $pass | cut -c9-13)
    timeout -s KILL 90 rocprofv3 --pmc $pass -d $O/$tag -o run --output-format csv -- python3 tools/traffic_probe.py --config c3 --raw $1 --out-align $2 > $O/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -3 $O/$tag.log; exit 1; }
    echo "$tag ok"
  done
done
