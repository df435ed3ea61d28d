#!/bin/bash
# Why the ChaCha open kernels read more than the seals (C5 planned open: 2x the 128-B reads): seal,
# open of the sealed records, and a second seal reading the first seal's output (same layout as the
# open), for C3 (direct) and C5 (planned); read and write request counts per kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; O=gpurun_out/traffic4; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for cfg in c3 c5; do
  for op in seal open reseal; do
    for pass in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
      tag=${cfg}_${op}_$(echo $pass | cut -c9-13)
      timeout -s KILL 90 rocprofv3 --pmc $pass -d $O/$tag -o run --output-format csv -- python3 tools/traffic_probe.py --config $cfg --op $op --steps 3 > $O/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -3 $O/$tag.log; exit 1; }
      echo "$tag ok $(tail -1 $O/$tag.log)"
    done
  done
done
