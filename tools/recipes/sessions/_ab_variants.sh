#!/bin/bash
# Parity of every variant library (config + parity tests), then interleaved same-box timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for lib in anothertls_amd/variants/libatls_*.so; do
  n=$(basename $lib .so); case $n in *dbg*) echo "$n: timing only"; continue;; esac
  ATLS_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_wire_mode.py > gpurun_out/par_$n.log 2>&1 || { echo "$n parity FAIL"; tail -20 gpurun_out/par_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/par_$n.log)"
done
for cfg in ${CONFIGS:-c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB}; do
for round in 1 2 3; do
  for lib in anothertls_amd/variants/libatls_*.so; do
    r=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])") || exit 1
    echo "$cfg round $round $(basename $lib .so): $r"
  done
done; done
