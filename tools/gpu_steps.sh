#!/bin/bash
# Run GPU steps on the gpurun box, each under its own time limit. Stops at the first step that
# faults, aborts or times out (exit codes other than 0/1); test failures (1) do not stop later steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local name=$1 limit=$2; shift 2
  echo "[$(date +%T)] start $name" >> gpurun_out/steps.log
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider ;;
    pytest_all) run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) run bench 600 python bench.py ;;
    bench_waves) for w in 4 8 12; do ATLS_GCM_WAVES=$w run bench_w$w 300 python bench.py --no-cpu-baseline; done ;;
    pmc_lds) export TMPDIR=/tmp; run pmc_lds 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_lds -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    variants) for lib in anothertls_amd/variants/libatls_nb*.so; do for w in 8 12 16; do t=$(basename $lib .so)_w$w; ATLS_LIB=$PWD/$lib ATLS_GCM_WAVES=$w run var_$t 300 python bench.py --no-cpu-baseline --steps 10; done; done ;;
    bench_tt) ATLS_GCM_BS=0 run bench_tt 300 python bench.py --no-cpu-baseline --steps 10 ;;
    bench_c4) run bench_c4 600 python bench.py --config c4_aes256gcm_1Mi_x_16KiB --records 65536 --no-cpu-baseline ;;
    pmc_bs) export TMPDIR=/tmp; run pmc_bs1 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_bs1 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline && \
            run pmc_bs2 600 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d gpurun_out/pmc_bs2 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    stamps) run stamps 300 python tools/bs_stamps.py ;;
    bs_debug) run bs_debug 120 python tools/bs_debug.py ;;
    bench_c3) run bench_c3 600 python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --no-cpu-baseline ;;
    bench_c5) run bench_c5 600 python bench.py --config c5_mixed_256Ki_x_64B-16KiB --no-cpu-baseline ;;
    prof) export TMPDIR=/tmp; run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    prof_c3) export TMPDIR=/tmp; run prof_c3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --steps 10 --warmup 2 --no-cpu-baseline ;;
    pmc) export TMPDIR=/tmp; run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline && \
         run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline && \
         run pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
