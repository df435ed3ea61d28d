#!/bin/bash
# Round 4 same-box A/B of library variants (anothertls_amd/variants/libatls_*.so, tools/build_variants.py):
# parity of every variant first (GCM / ChaCha parity, planned batches, wire mode and the full-size configs),
# then CONFIGS x variants interleaved over ROUNDS rounds: bench.py seal + open kernel ms (HIP events).
# Usage: VARIANTS="base fastfirst" CONFIGS="c5_mixed_256Ki_x_64B-16KiB c2_aes128gcm_64Ki_x_16KiB" ROUNDS=3 bash tools/recipes/r4_ab.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag=$1
out=gpurun_out/r4/ab_$tag.log
mkdir -p gpurun_out/r4
: > $out
for lib in $(for v in ${VARIANTS:-base}; do echo anothertls_amd/variants/libatls_$v.so; done); do
  v=$(basename $lib .so)
  ATLS_LIB=$PWD/$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan.py tests/test_wire_mode.py tests/test_gpu_chacha_widths.py tests/test_gpu_configs.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4/ab_${tag}_parity_$v.txt 2>&1 || { echo "$v parity FAILED" >> $out; tail -30 gpurun_out/r4/ab_${tag}_parity_$v.txt; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/r4/ab_${tag}_parity_$v.txt)" >> $out
done
for round in $(seq 1 ${ROUNDS:-3}); do
  for cfg in ${CONFIGS:-c5_mixed_256Ki_x_64B-16KiB}; do
    for lib in $(for v in ${VARIANTS:-base}; do echo anothertls_amd/variants/libatls_$v.so; done); do
      r=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --no-configs --sustain-s 0 --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['open']['kernel_ms'], d['open']['plaintext_and_status_ok'])") || exit $?
      echo "round $round $cfg $(basename $lib .so): GiBps seal_ms frac open_ms ok = $r" >> $out
    done
  done
done
cat $out
