#!/bin/bash
# C5 (mixed suites, ChaCha kernel beside the AES-GCM kernel): variants x ChaCha workgroups per CU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for lib in anothertls_amd/variants/libatls_*.so; do
  n=$(basename $lib .so)
  ATLS_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_chacha_widths.py > gpurun_out/par_$n.log 2>&1 || { echo "$n parity FAIL"; tail -20 gpurun_out/par_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/par_$n.log)"
done
for round in 1 2; do
  for lib in anothertls_amd/variants/libatls_*.so; do
    n=$(basename $lib .so)
    for w in ${WGS:-1 2 4 8}; do
      r=$(ATLS_CHACHA_WGS=$w ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config c5_mixed_256Ki_x_64B-16KiB --no-cpu-baseline --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])") || exit 1
      echo "round $round $n wgs=$w c5: $r"
    done
    r=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --no-cpu-baseline --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])") || exit 1
    echo "round $round $n c3: $r"
  done
done
