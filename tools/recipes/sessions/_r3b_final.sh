#!/bin/bash
# Round 3, second session, final measurement pass on one box. A: GPU tests, smoke, bench lines C1-C5
# (C2 with the CPU baseline, host-memory and wire rates), single-call latency. B: rocprofv3 stats and
# FETCH / WRITE PMC of C3 (its kernels changed this session; tools/profile_round.sh) and the wave-state
# PMC of the C3 kernels. Stops at the first step that faults, aborts or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out/final
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/final
run() { local n=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$n.log 2>&1 || { echo "$n failed rc=$?"; tail -5 $O/$n.log; exit 1; }; echo "$n: $(tail -1 $O/$n.log | cut -c1-240)"; }
case ${1:-A} in
  A)
    run tests 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
    run c2 400 python bench.py --pcie --wire
    run c3 300 python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --no-cpu-baseline
    run c4 300 python bench.py --config c4_aes256gcm_1Mi_x_16KiB --no-cpu-baseline
    run c5 300 python bench.py --config c5_mixed_256Ki_x_64B-16KiB --no-cpu-baseline
    run c1 300 python bench.py --config c1_server_https_loopback_1MiB --steps 20
    run single 300 python tools/single_call_latency.py
    ;;
  C)  # C2 / C4 / C5 bench lines and their rocprof stats + FETCH / WRITE PMC on the same box
    run c2 400 python bench.py --pcie --wire
    run c4 300 python bench.py --config c4_aes256gcm_1Mi_x_16KiB --no-cpu-baseline
    run c5 300 python bench.py --config c5_mixed_256Ki_x_64B-16KiB --no-cpu-baseline
    for c in c2:c2_aes128gcm_64Ki_x_16KiB c4:c4_aes256gcm_1Mi_x_16KiB c5:c5_mixed_256Ki_x_64B-16KiB; do
      bash tools/profile_round.sh ${c#*:} ${c%%:*} || exit 1
    done
    bash tools/pmc_stall.sh c2_aes128gcm_64Ki_x_16KiB > $O/pmc_c2.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
    echo "C done"
    ;;
  B)
    bash tools/profile_round.sh c3_chacha20poly1305_64Ki_x_1.5KiB c3 || exit 1
    bash tools/pmc_stall.sh c3_chacha20poly1305_64Ki_x_1.5KiB > $O/pmc_c3.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
    echo "B done"
    ;;
esac
