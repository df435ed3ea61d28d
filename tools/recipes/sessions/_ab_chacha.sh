#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for lib in anothertls_amd/variants/libatls_*.so; do
  n=$(basename $lib .so)
  ATLS_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_chacha_widths.py tests/test_gpu_configs.py::test_c5_shard_full_vs_oracle_and_openssl tests/test_gpu_plan.py tests/test_wire_mode.py -k "not sticky" > gpurun_out/par_$n.log 2>&1 || { echo "$n parity FAIL"; tail -20 gpurun_out/par_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/par_$n.log)"
done
for round in 1 2 3; do
  for lib in anothertls_amd/variants/libatls_*.so; do
    n=$(basename $lib .so)
    c3=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])") || exit 1
    c5=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config c5_mixed_256Ki_x_64B-16KiB --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])") || exit 1
    op=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python tools/open_bench.py 2>/dev/null | tail -1) || exit 1
    echo "round $round $n: C3 $c3 | C5 $c5 | C3 open $op"
  done
done
