#!/bin/bash
# Round 5 same-box A/B of library variants (anothertls_amd/variants/libatls_*.so, tools/build_variants.py).
# PARITY=1: the parity suites on every variant first (skip for ATLS_DBG_* timing builds, whose results are wrong
# on purpose). Then CONFIGS x variants interleaved over ROUNDS rounds: bench.py seal + open kernel ms.
# BENCH_ARGS: extra bench.py flags (e.g. "--key-slots 65536": C2 with a key per record).
# Usage: VARIANTS="base skip1" CONFIGS="c2_aes128gcm_64Ki_x_16KiB" ROUNDS=3 bash tools/recipes/r5_ab.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out/r5
out=gpurun_out/r5/ab_$tag.log
: > $out
if [ "${PARITY:-1}" = 1 ]; then
  for v in ${VARIANTS:-base}; do
    lib=anothertls_amd/variants/libatls_$v.so
    ATLS_LIB=$PWD/$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan.py tests/test_wire_mode.py tests/test_gpu_gcm_groups.py tests/test_gpu_configs.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5/ab_${tag}_parity_$v.txt 2>&1 || { echo "$v parity FAILED" >> $out; tail -30 gpurun_out/r5/ab_${tag}_parity_$v.txt; exit 1; }
    echo "$v parity: $(tail -1 gpurun_out/r5/ab_${tag}_parity_$v.txt)" >> $out
  done
fi
for round in $(seq 1 ${ROUNDS:-3}); do
  for cfg in ${CONFIGS:-c2_aes128gcm_64Ki_x_16KiB}; do
    for v in ${VARIANTS:-base}; do
      lib=anothertls_amd/variants/libatls_$v.so
      r=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --no-configs --sustain-s 0 --steps 20 ${BENCH_ARGS:-} 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); l=d['roofline'].get('lds') or {}; print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], l.get('sclk_MHz'), d['open']['kernel_ms'], d['open']['plaintext_and_status_ok'])") || exit $?
      echo "round $round $cfg $v: GiBps seal_ms frac sclk open_ms ok = $r" >> $out
    done
  done
done
cat $out
