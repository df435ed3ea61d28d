#!/bin/bash
# ChaCha LDS carry A/B: parity per variant, C3 / C5 bench lines interleaved (3 rounds), then C3
# FETCH / WRITE per variant (seal and open kernels of the bench run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; O=gpurun_out/carry; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
TESTS="tests/test_gpu_chacha_widths.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_wire_mode.py" CONFIGS="c3_chacha20poly1305_64Ki_x_1.5KiB c5_mixed_256Ki_x_64B-16KiB" BENCH_EXTRA=" " PMC=0 bash tools/recipes/sessions/_ab_r3.sh || exit $?
for lib in anothertls_amd/variants/libatls_*.so; do
  n=$(basename $lib .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    ATLS_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $c -d $O/${n}_$c -o run --output-format csv -- python3 bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --steps 5 --warmup 2 --no-cpu-baseline > $O/${n}_$c.log 2>&1 || { echo "pmc $n $c rc=$?"; exit 1; }
  done
  echo "pmc $n done"
done
