#!/bin/bash
# Request sizes behind FETCH_SIZE / WRITE_SIZE for the seal and open kernels of C3 and C5: the
# memory-side read requests split by size (128 / 64 / 32 B), writes (all / 64 B) and the DRAM part of
# both, two TCC counters per pass (MI355X_MICROARCH.md: calibrate uncalibrated access patterns).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; O=gpurun_out/reqsize; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for cfg in c3:c3_chacha20poly1305_64Ki_x_1.5KiB c5:c5_mixed_256Ki_x_64B-16KiB; do
  i=0
  for pass in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" \
              "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"; do
    i=$((i+1)); tag=${cfg%%:*}_p$i
    timeout -s KILL 90 rocprofv3 --pmc $pass -d $O/$tag -o run --output-format csv -- python3 bench.py --config ${cfg#*:} --steps 5 --warmup 2 --no-cpu-baseline > $O/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -3 $O/$tag.log; exit 1; }
    echo "$tag ok"
  done
done
