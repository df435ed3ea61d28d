#!/bin/bash
# Round 4: C5 re-sweep after the LDS lane combine and the spread work list: AES-GCM waves per workgroup
# (ATLS_GCM_WAVES) x ChaCha20-Poly1305 workgroups per CU (ATLS_CHACHA_WGS), and the planned ChaCha lane
# width (variant g8 = -DATLS_CHACHA_PLANNED_G=8), interleaved over 3 rounds; seal / open kernel ms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r4/c5_sweep.log
mkdir -p gpurun_out/r4
: > $out
cfg=c5_mixed_256Ki_x_64B-16KiB
run() {  # label, env..., lib
  local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --no-configs --sustain-s 0 --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['open']['kernel_ms'], d['open']['plaintext_and_status_ok'])") || exit 1
  echo "round $round $label: GiBps seal_ms frac open_ms ok = $r" >> $out
}
ATLS_LIB=$PWD/anothertls_amd/variants/libatls_g8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_plan.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4/c5_sweep_parity_g8.txt 2>&1 || { tail -20 gpurun_out/r4/c5_sweep_parity_g8.txt; exit 1; }
echo "g8 parity: $(tail -1 gpurun_out/r4/c5_sweep_parity_g8.txt)" >> $out
for round in 1 2 3; do
  for w in 12 8; do
    for c in 8 4 16; do
      run "waves$w wgs$c" ATLS_GCM_WAVES=$w ATLS_CHACHA_WGS=$c
    done
  done
  run "g8 waves12 wgs8" ATLS_LIB=$PWD/anothertls_amd/variants/libatls_g8.so
done
cat $out
