#!/bin/bash
# Round 5: bracket the RCCL point-to-point size defect for both RCCLs of the image (tools/rccl_p2p_probe), then
# the multi-engine tests (the 1 GiB cap just under / at / over) and the clock / power study.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5rccl; mkdir -p $O
TL=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib', 'librccl.so'))")
G=1073741824
SIZES="$((G-4096)) $G $((G+4096)) $((G+16777216)) $((G+268435456)) $((G+536870912)) $((2*G-4096)) $((2*G))"
# timeout -k 10 300 tools/rccl_p2p_probe $TL $SIZES > $O/rccl_p2p_probe_torch.log 2>&1 || { tail -20 $O/rccl_p2p_probe_torch.log; exit 1; }
# cat $O/rccl_p2p_probe_torch.log
# timeout -k 10 300 tools/rccl_p2p_probe /opt/rocm/lib/librccl.so.1 $SIZES > $O/rccl_p2p_probe_rocm.log 2>&1 || { tail -20 $O/rccl_p2p_probe_rocm.log; exit 1; }
# cat $O/rccl_p2p_probe_rocm.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_dist.txt 2>&1 || { tail -30 $O/gpu_tests_dist.txt; exit 1; }
tail -1 $O/gpu_tests_dist.txt
grep -h "anothertls_amd: RCCL" $O/gpu_tests_dist.txt | head -2
timeout -k 10 300 python -u tools/clock_power.py --seconds 8 > $O/clock_power.json 2> $O/clock_power.err || { tail -30 $O/clock_power.err; exit 1; }
tail -8 $O/clock_power.err
