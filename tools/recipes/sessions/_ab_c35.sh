#!/bin/bash
# Same-box A/B of anothertls_amd/variants/libatls_*.so on C3 and C5 (seal and open kernels): ChaCha parity
# per variant (widths vs the oracle, full C3 batch vs OpenSSL, the C5 shard vs the oracle, plan and wire
# tests), then 3 interleaved rounds of the C3 and C5 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for lib in anothertls_amd/variants/libatls_*.so; do
  n=$(basename $lib .so)
  ATLS_LIB=$PWD/$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_chacha_widths.py tests/test_gpu_configs.py::test_c3_full_batch_device_resident_vs_openssl_and_oracle tests/test_gpu_configs.py::test_c5_shard_full_vs_oracle_and_openssl tests/test_gpu_plan.py tests/test_wire_mode.py -k "not sticky" -p no:cacheprovider > gpurun_out/par_$n.log 2>&1 || { echo "$n parity FAIL"; tail -20 gpurun_out/par_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/par_$n.log)"
done
for round in 1 2 3; do
  for lib in anothertls_amd/variants/libatls_*.so; do
    n=$(basename $lib .so)
    for c in c3_chacha20poly1305_64Ki_x_1.5KiB c5_mixed_256Ki_x_64B-16KiB; do
      r=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config $c --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'seal', d['roofline']['kernel_ms'], 'open', d['open']['kernel_ms'])") || exit 1
      echo "round $round $n ${c%%_*}: $r"
    done
  done
done
