#!/bin/bash
# Round-2 measurement pass on one box: bench lines for C1-C5 (+ PCIe-inclusive and wire rates on C2),
# then rocprofv3 kernel-trace stats and FETCH/WRITE PMC passes per config (tools/profile_round.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1; shift; timeout -k 10 400 "$@" > gpurun_out/m_$n.log 2>&1 || { echo "$n failed rc=$?"; tail -5 gpurun_out/m_$n.log; exit 1; }; echo "$n: $(tail -1 gpurun_out/m_$n.log | cut -c1-400)"; }
run c2 python bench.py --pcie --wire
run c3 python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --no-cpu-baseline
run c4 python bench.py --config c4_aes256gcm_1Mi_x_16KiB --no-cpu-baseline
run c5 python bench.py --config c5_mixed_256Ki_x_64B-16KiB --no-cpu-baseline
run c1 python bench.py --config c1_server_https_loopback_1MiB --steps 20
for c in c2:c2_aes128gcm_64Ki_x_16KiB c3:c3_chacha20poly1305_64Ki_x_1.5KiB c4:c4_aes256gcm_1Mi_x_16KiB c5:c5_mixed_256Ki_x_64B-16KiB; do
  bash tools/profile_round.sh ${c#*:} ${c%%:*} || exit 1
done
