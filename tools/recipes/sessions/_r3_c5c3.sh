#!/bin/bash
# C5 lazy-join A/B (same box, interleaved, 3 rounds) and C3 traffic probes (TCC request-size
# counters of the ChaCha kernel next to C2's AES-GCM kernel). Stops at the first fault or timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out/c5c3
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/c5c3
C5=c5_mixed_256Ki_x_64B-16KiB; C3=c3_chacha20poly1305_64Ki_x_1.5KiB
val() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d.get('open',{}).get('kernel_ms'))"; }
if [ -z "$SKIP_AB" ]; then
for round in 1 2 3; do
  for mode in lazy joined; do
    extra=""; [ $mode = joined ] && extra="--no-lazy-join"
    timeout -k 10 120 python bench.py --config $C5 --no-cpu-baseline $extra > $O/b.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/b.log; exit 1; }
    echo "round $round c5 $mode: $(val $O/b.log)"
  done
done
fi
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
grep -oE "TCC_EA0?_(RD|WR)REQ[A-Z0-9_]*" $O/counters.txt | sort -u | tr '\n' ' '; echo
for cfg in $C3 c2_aes128gcm_64Ki_x_16KiB; do
  CMD="python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-open"
  for pass in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    tag=$(echo $pass | cut -c1-14 | tr ' ' '_')
    timeout -s KILL 90 rocprofv3 --pmc $pass -d $O/pmc_${cfg:0:2}_$tag -o run --output-format csv -- $CMD > $O/pmc_${cfg:0:2}_$tag.log 2>&1 || { echo "pmc $cfg $pass rc=$?"; tail -3 $O/pmc_${cfg:0:2}_$tag.log; }
  done
done
echo done
