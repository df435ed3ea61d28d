#!/bin/bash
# Same-box A/B of anothertls_amd/variants/libatls_*.so for the GCM general steps: parity (GCM groups,
# full-size configs, wire, parity, plan tests), then C5 / C2 / C4 seal+open kernel times, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for lib in anothertls_amd/variants/libatls_*.so; do
  n=$(basename $lib .so)
  ATLS_LIB=$PWD/$lib timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gcm_groups.py tests/test_gpu_configs.py tests/test_wire_mode.py tests/test_gpu_parity.py tests/test_gpu_plan.py -k "not sticky" -p no:cacheprovider > gpurun_out/par_$n.log 2>&1 || { echo "$n parity FAIL"; tail -20 gpurun_out/par_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/par_$n.log)"
done
for round in 1 2 3; do
  for lib in anothertls_amd/variants/libatls_*.so; do
    n=$(basename $lib .so)
    for c in c5_mixed_256Ki_x_64B-16KiB c2_aes128gcm_64Ki_x_16KiB; do
      r=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config $c --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'seal', d['roofline']['kernel_ms'], 'open', d['open']['kernel_ms'])") || exit 1
      echo "round $round $n ${c%%_*}: $r"
    done
  done
done
