#!/bin/bash
# T-table rows written 16 B per store (ATLS_TT_B128, default) against one word per store (tt0): parity of the
# default build, then single-call floors and the C2 / C4 bench kernels per variant, 3 interleaved rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5tt; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gcm_groups.py tests/test_gpu_single_call.py tests/test_gpu_single_resident.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/parity.txt 2>&1 || { tail -30 $O/parity.txt; exit 1; }
tail -1 $O/parity.txt
for r in 1 2 3; do
  for v in base tt0; do
    LD_LIBRARY_PATH=$PWD/anothertls_amd/variants/d_$v timeout -k 10 120 ./tools/single_call_floor > $O/floor_${v}_$r.json 2>&1 || { tail -5 $O/floor_${v}_$r.json; exit 1; }
    python3 -c "import json; d=json.load(open('$O/floor_${v}_$r.json')); print('round $r $v', {k: d[k] for k in ('aes128gcm_1537_seal_us','aes128gcm_1537_open_us','aes128gcm_16385_seal_us')})"
    for cfg in c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB; do
      ATLS_LIB=$PWD/anothertls_amd/variants/d_$v/libatls.so timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --no-configs --sustain-s 0 --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('round $r $v $cfg', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['open']['kernel_ms'])" || exit 1
    done
  done
done
