#!/bin/bash
# Opens keeping the last non-zero plaintext block per lane (ATLS_OPEN_NZ_KEEP, default) against the per-block
# scan (nz0): every GPU test on the default build, then bench seal / open kernels per variant, 3 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5nz; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
for r in 1 2 3; do
  for v in base nz0; do
    for cfg in c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB c5_mixed_256Ki_x_64B-16KiB; do
      ATLS_LIB=$PWD/anothertls_amd/variants/d_$v/libatls.so timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --no-configs --sustain-s 0 --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('round $r $v $cfg seal', d['roofline']['kernel_ms'], 'open', d['open']['kernel_ms'], d['open']['frac'], d['open']['plaintext_and_status_ok'])" || exit 1
    done
    ATLS_LIB=$PWD/anothertls_amd/variants/d_$v/libatls.so timeout -k 10 120 python bench.py --config c2_aes128gcm_64Ki_x_16KiB --key-slots 65536 --no-cpu-baseline --no-configs --sustain-s 0 --steps 10 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('round $r $v c2-keyrec seal', d['roofline']['kernel_ms'], 'open', d['open']['kernel_ms'], d['open']['frac'], d['open']['plaintext_and_status_ok'])" || exit 1
  done
done
