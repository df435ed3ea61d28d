#!/bin/bash
# ChaCha open register pressure A/B: MAC before keystream (planned opens / all opens) and a 3-wave
# bound for the planned open kernel, against the current build. Parity, C3 / C5 seal + open lines
# over 3 interleaved rounds, then C5 read / write request counts per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; O=gpurun_out/macfirst; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
TESTS="tests/test_gpu_chacha_widths.py tests/test_gpu_parity.py tests/test_gpu_plan.py tests/test_wire_mode.py" CONFIGS="c3_chacha20poly1305_64Ki_x_1.5KiB c5_mixed_256Ki_x_64B-16KiB" BENCH_EXTRA=" " PMC=0 bash tools/recipes/sessions/_ab_r3.sh || exit $?
for lib in anothertls_amd/variants/libatls_*.so; do
  n=$(basename $lib .so)
  for pass in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    tag=${n}_$(echo $pass | cut -c9-13)
    ATLS_LIB=$PWD/$lib timeout -s KILL 90 rocprofv3 --pmc $pass -d $O/$tag -o run --output-format csv -- python3 tools/traffic_probe.py --config c5 --op open --steps 3 > $O/$tag.log 2>&1 || { echo "pmc $tag rc=$?"; tail -3 $O/$tag.log; exit 1; }
  done
  echo "pmc $n done"
done
