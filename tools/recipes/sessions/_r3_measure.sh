#!/bin/bash
# Round-3 measurement pass on one box. Part A: GPU tests, smoke, bench lines C1-C5 (C2 with the CPU
# baseline, PCIe-inclusive and wire rates). Part B: rocprofv3 kernel-trace stats and FETCH / WRITE
# PMC per config (tools/profile_round.sh), wave-state PMC of the C2 kernel (tools/pmc_stall.sh).
# Stops at the first step that faults, aborts or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/m_$n.log 2>&1 || { echo "$n failed rc=$?"; tail -5 gpurun_out/m_$n.log; exit 1; }; echo "$n: $(tail -1 gpurun_out/m_$n.log | cut -c1-300)"; }
case ${1:-A} in
  A)
    run tests 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
    run c2 400 python bench.py --pcie --wire
    run c3 300 python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --no-cpu-baseline
    run c4 300 python bench.py --config c4_aes256gcm_1Mi_x_16KiB --no-cpu-baseline
    run c5 300 python bench.py --config c5_mixed_256Ki_x_64B-16KiB --no-cpu-baseline
    run c1 300 python bench.py --config c1_server_https_loopback_1MiB --steps 20
    ;;
  B)
    for c in ${CFGS:-c2:c2_aes128gcm_64Ki_x_16KiB c3:c3_chacha20poly1305_64Ki_x_1.5KiB c4:c4_aes256gcm_1Mi_x_16KiB c5:c5_mixed_256Ki_x_64B-16KiB}; do
      bash tools/profile_round.sh ${c#*:} ${c%%:*} || exit 1
    done
    [ -n "$CFGS" ] || bash tools/pmc_stall.sh c2_aes128gcm_64Ki_x_16KiB || exit 1
    ;;
esac
