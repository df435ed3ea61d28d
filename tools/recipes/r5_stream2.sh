#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5st2; mkdir -p $O
for a in "8 64 1" "8 64 8" "2 256 8"; do ATLS_SB_PROFILE=1 timeout -k 10 120 tools/c1_loopback_native $a || exit 1; done > $O/c1_scale_profile.log 2>&1
cat $O/c1_scale_profile.log
nproc; cat /proc/cpuinfo | grep "model name" | head -1; taskset -p $$ || true; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
