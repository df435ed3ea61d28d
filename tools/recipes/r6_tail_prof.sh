#!/bin/bash
# Round 6: rocprof kernel trace of C2 with a key per record, deferred tails on and off (ATLS_GCM_TAIL_ON).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r6d}
mkdir -p $O
for on in 1 0; do
  ATLS_GCM_TAIL_ON=$on timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$on -o run --output-format csv -- \
    python3 bench.py --config c2_aes128gcm_64Ki_x_16KiB --key-slots 65536 --no-cpu-baseline --no-configs --sustain-s 0 --steps 20 --no-open \
    > $O/bench_$on.json 2> $O/bench_$on.err || { tail -20 $O/bench_$on.err; exit 1; }
  f=$(ls $O/prof_$on/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls $O/prof_$on/run_kernel_stats.csv)
  echo "== tail_on=$on"; cut -c1-200 $f | head -12
done
