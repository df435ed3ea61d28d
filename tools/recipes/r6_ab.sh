#!/bin/bash
# Round 6 same-box A/B of library variants (anothertls_amd/variants/libatls_*.so, tools/build_variants.py).
# PARITY=1: the parity suites on every variant first (skip for ATLS_DBG_* timing builds, whose results are wrong
# on purpose). Then CONFIGS x variants interleaved over ROUNDS rounds: bench.py seal + open kernel ms and the
# same-window clock. A config token is name[:records[:key_slots]] (records 0 = the config's per-GPU shard).
# Usage: VARIANTS="base minw1" CONFIGS="c5_mixed_256Ki_x_64B-16KiB:262144" ROUNDS=3 bash tools/recipes/r6_ab.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag=$1
mkdir -p ${O:-gpurun_out/r6}
out=${O:-gpurun_out/r6}/ab_$tag.log
: > $out
if [ "${PARITY:-1}" = 1 ]; then
  for v in ${VARIANTS:-base}; do
    lib=anothertls_amd/variants/libatls_$v.so
    ATLS_LIB=$PWD/$lib timeout -k 10 500 python -u -m pytest ${PARITY_TESTS:-tests/test_gpu_parity.py tests/test_gpu_plan.py tests/test_wire_mode.py tests/test_gpu_gcm_groups.py tests/test_gpu_configs.py} -x -q -m gpu --timeout 300 --timeout-method thread > ${O:-gpurun_out/r6}/ab_${tag}_parity_$v.txt 2>&1 || { echo "$v parity FAILED" >> $out; tail -30 ${O:-gpurun_out/r6}/ab_${tag}_parity_$v.txt; exit 1; }
    echo "$v parity: $(tail -1 ${O:-gpurun_out/r6}/ab_${tag}_parity_$v.txt)" >> $out
  done
fi
for round in $(seq 1 ${ROUNDS:-3}); do
  for tok in ${CONFIGS:-c2_aes128gcm_64Ki_x_16KiB}; do
    IFS=: read -r cfg recs keys <<< "$tok"
    extra=""
    [ -n "${recs:-}" ] && [ "$recs" != 0 ] && extra="$extra --records $recs"
    [ -n "${keys:-}" ] && extra="$extra --key-slots $keys"
    for v in ${VARIANTS:-base}; do
      lib=anothertls_amd/variants/libatls_$v.so
      r=$(ATLS_LIB=$PWD/$lib timeout -k 10 150 python bench.py --config $cfg --no-cpu-baseline --no-configs --sustain-s 0 --steps 20 $extra ${BENCH_ARGS:-} 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); l=d['roofline'].get('lds') or {}; o=d['open']; print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], l.get('sclk_MHz'), l.get('frac'), o['kernel_ms'], o['frac'], o['plaintext_and_status_ok'])") || exit $?
      echo "round $round $tok $v: GiBps seal_ms frac sclk lds_frac open_ms open_frac ok = $r" >> $out
    done
  done
done
cat $out
