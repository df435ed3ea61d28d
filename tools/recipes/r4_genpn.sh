#!/bin/bash
# Round 4: the last general step from the fast step's prefetch (ATLS_GEN_PN) -- parity of both builds
# (GCM parity, wire mode, plan, configs incl. the whole C5 shard vs the oracle, groups), batch phase clocks,
# then C5, C2 with a key per record and C2 interleaved over 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
out=gpurun_out/r4/ab_genpn.log
: > $out
for v in base genpn; do
  ATLS_LIB=$PWD/anothertls_amd/variants/libatls_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan.py tests/test_wire_mode.py tests/test_gpu_configs.py tests/test_gpu_gcm_groups.py tests/test_gpu_single_call.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4/ab_genpn_parity_$v.txt 2>&1 || { echo "$v parity FAILED" >> $out; tail -30 gpurun_out/r4/ab_genpn_parity_$v.txt; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/r4/ab_genpn_parity_$v.txt)" >> $out
done
bash tools/recipes/r4_ttb.sh > /dev/null 2>&1 || exit 1
cp gpurun_out/r4/tt_batch.log gpurun_out/r4/tt_batch_genpn.log
for round in 1 2 3; do
  for a in "c5_mixed_256Ki_x_64B-16KiB" "c2_aes128gcm_64Ki_x_16KiB --key-slots 65536" "c2_aes128gcm_64Ki_x_16KiB"; do
    for v in base genpn; do
      r=$(ATLS_LIB=$PWD/anothertls_amd/variants/libatls_$v.so timeout -k 10 120 python bench.py --config $a --no-cpu-baseline --no-configs --sustain-s 0 --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['open']['kernel_ms'], d['open']['plaintext_and_status_ok'])") || exit 1
      echo "round $round $a $v: GiBps seal_ms frac open_ms ok = $r" >> $out
    done
  done
done
cat $out gpurun_out/r4/tt_batch_genpn.log
