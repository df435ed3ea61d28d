#!/bin/bash
# Same-box A/B of anothertls_amd/variants/libatls_*.so on C3 (ChaCha20-Poly1305 seal and open kernels):
# ChaCha parity per variant (widths vs the oracle, the full C3 batch device-resident vs OpenSSL, wire and
# planned batches), then 3 interleaved rounds of the C3 bench line (seal and open kernel ms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for lib in anothertls_amd/variants/libatls_*.so; do
  n=$(basename $lib .so)
  ATLS_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chacha_widths.py tests/test_gpu_configs.py::test_c3_full_batch_device_resident_vs_openssl_and_oracle tests/test_gpu_plan.py tests/test_wire_mode.py -k "not sticky" -p no:cacheprovider > gpurun_out/par_$n.log 2>&1 || { echo "$n parity FAIL"; tail -20 gpurun_out/par_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/par_$n.log)"
done
for round in 1 2 3; do
  for lib in anothertls_amd/variants/libatls_*.so; do
    n=$(basename $lib .so)
    r=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'seal', d['roofline']['kernel_ms'], 'open', d['open']['kernel_ms'], d['open'].get('GiBps'))") || exit 1
    echo "round $round $n: C3 $r"
  done
done
