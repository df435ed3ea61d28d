#!/bin/bash
# Round 6: C3's launch and per-record floor. Timing builds (no parity): base, dbg7 (no keystream, MAC or full-block
# memory), dbg128 (each wave reads its step's record lengths and exits); bench HIP events and a rocprof kernel trace
# of each (kernel duration without the gaps between launches). Outputs under gpurun_out/r6f/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r6f}
mkdir -p $O
O=$O PARITY=0 VARIANTS="${VARIANTS:-base dbg7 dbg128}" CONFIGS="c3_chacha20poly1305_64Ki_x_1.5KiB" ROUNDS=2 bash tools/recipes/r6_ab.sh c3floor || exit 1
for v in ${VARIANTS:-base dbg7 dbg128}; do
  ATLS_LIB=$PWD/anothertls_amd/variants/libatls_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- \
    python3 bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --no-cpu-baseline --no-configs --sustain-s 0 --steps 20 --no-open > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  f=$(ls $O/prof_$v/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls $O/prof_$v/run_kernel_stats.csv)
  echo "== $v"; grep -i chacha $f | cut -c1-220
done
