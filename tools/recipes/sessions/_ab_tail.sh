#!/bin/bash
# Same-box A/B of the grouped batch's tail policy over record counts (C2 records, 16 KiB).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
for lib in anothertls_amd/variants/libatls_*.so; do
  n=$(basename $lib .so)
  ATLS_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gcm_groups.py tests/test_gpu_configs.py > gpurun_out/par_$n.log 2>&1 || { echo "$n parity FAIL"; tail -20 gpurun_out/par_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/par_$n.log)"
done
for round in 1 2; do
  for lib in anothertls_amd/variants/libatls_*.so; do
    n=$(basename $lib .so)
    for recs in 32768 65536 98304; do
      r=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --records $recs --no-cpu-baseline --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])") || exit 1
      echo "round $round $n records=$recs: $r"
    done
  done
done
