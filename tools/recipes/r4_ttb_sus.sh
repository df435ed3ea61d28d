#!/bin/bash
# Round 4: batch phase clocks (tools/recipes/r4_ttb.sh), then the bench's headline line with the sustained
# 5-second leg (bench.py --sustain-s) on C2 and C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/recipes/r4_ttb.sh || exit 1
timeout -k 10 200 python -u bench.py --no-configs --no-cpu-baseline > gpurun_out/r4/bench_sustained_c2.json 2> gpurun_out/r4/bench_sustained_c2.err || { tail -20 gpurun_out/r4/bench_sustained_c2.err; exit 1; }
timeout -k 10 200 python -u bench.py --config c5_mixed_256Ki_x_64B-16KiB --no-configs --no-cpu-baseline > gpurun_out/r4/bench_sustained_c5.json 2> gpurun_out/r4/bench_sustained_c5.err || { tail -20 gpurun_out/r4/bench_sustained_c5.err; exit 1; }
cat gpurun_out/r4/bench_sustained_c2.json gpurun_out/r4/bench_sustained_c5.json
