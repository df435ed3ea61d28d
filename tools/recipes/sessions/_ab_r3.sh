#!/bin/bash
# Same-box A/B of anothertls_amd/variants/libatls_*.so: parity per variant (grouped-path tests and the
# full-size configs), C2 / C4 bench lines interleaved over 3 rounds, then one wave-state PMC pass per
# variant on C2 (LDS array busy, LDS issue stalls, waits). Stops at the first fault or timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for lib in anothertls_amd/variants/libatls_*.so; do
  n=$(basename $lib .so)
  ATLS_LIB=$PWD/$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    ${TESTS:-tests/test_gpu_gcm_groups.py tests/test_gpu_configs.py} -p no:cacheprovider > gpurun_out/ab/par_$n.log 2>&1
  rc=$?; echo "$n parity rc=$rc: $(tail -1 gpurun_out/ab/par_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
for round in 1 2 3; do
  for lib in anothertls_amd/variants/libatls_*.so; do
    n=$(basename $lib .so)
    for cfg in ${CONFIGS:-c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB}; do
      ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline ${BENCH_EXTRA:---no-open} > gpurun_out/ab/b.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/ab/b.log; exit 1; }
      r=$(tail -1 gpurun_out/ab/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d.get('open', {}).get('kernel_ms'))")
      echo "round $round $n $cfg: $r"
    done
  done
done
if [ "${PMC:-1}" = 1 ]; then
  CMD="python3 bench.py --config ${PMC_CFG:-c2_aes128gcm_64Ki_x_16KiB} --steps 5 --warmup 2 --no-cpu-baseline --no-open"
  for lib in anothertls_amd/variants/libatls_*.so; do
    n=$(basename $lib .so)
    ATLS_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY ${PMC_EXTRA:-SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE} SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
      -d gpurun_out/ab/pmc_$n -o run --output-format csv -- $CMD > gpurun_out/ab/pmc_$n.log 2>&1 || { echo "pmc $n rc=$?"; exit 1; }
    echo "pmc $n done"
  done
fi
