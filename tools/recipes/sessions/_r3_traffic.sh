#!/bin/bash
# Write / read request counts of the record kernels for packed vs line-aligned layouts and 4096 vs 1
# keys (tools/traffic_probe.py under rocprofv3 --pmc, one counter group per pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; O=gpurun_out/traffic; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for v in "c3 16 4096" "c3 128 4096" "c3 16 1" "c3 128 1" "c2 16 4096" "c2 128 4096"; do
  set -- $v
  for pass in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    tag=$1_o$2_k$3_$(echo $pass | cut -c9-13)
    timeout -s KILL 90 rocprofv3 --pmc $pass -d $O/$tag -o run --output-format csv -- python3 tools/traffic_probe.py --config $1 --out-align $2 --keys $3 > $O/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -3 $O/$tag.log; exit 1; }
    echo "$tag ok"
  done
done
