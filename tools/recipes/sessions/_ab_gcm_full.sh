#!/bin/bash
# Same-box A/B of AES-GCM library variants (anothertls_amd/variants/libatls_*.so) with the full-size
# parity tests: grouped-path tests, the parity suite and the C2 / C4 / C5 config checks per variant,
# then C2 / C4 bench lines, interleaved, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for lib in anothertls_amd/variants/libatls_*.so; do
  n=$(basename $lib .so)
  ATLS_LIB=$PWD/$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gcm_groups.py tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/par_$n.log 2>&1 || { echo "$n parity FAIL"; tail -20 gpurun_out/par_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/par_$n.log)"
done
for round in 1 2 3; do
  for lib in anothertls_amd/variants/libatls_*.so; do
    n=$(basename $lib .so)
    for cfg in ${CONFIGS:-c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB}; do
      r=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])") || exit 1
      echo "round $round $n $cfg: $r"
    done
  done
done
