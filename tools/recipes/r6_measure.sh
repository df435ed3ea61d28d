#!/bin/bash
# Round 6 final measurement pass on one box: every GPU test, the smoke, the default bench line (C2 with roofline.lds + the
# C3 / C4 / C5 shards, C2 with a key per record, C4 and C5 whole), C2's PCIe-inclusive and wire rates, C1 (with the
# at-scale runs), rocprof kernel traces and FETCH_SIZE / WRITE_SIZE passes of every config (tools/profile_round.sh
# -> kstats.py here, traffic.py after), the key-install timings under rocprof and the single-call floors (launch
# path and resident server). Outputs under gpurun_out/r6m/ (O=... overrides).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r6m}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 300 python -u bench.py --pcie --wire --no-configs --no-cpu-baseline > $O/bench_c2_pcie_wire.json 2> $O/bench_c2_pcie_wire.err || { tail -20 $O/bench_c2_pcie_wire.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c1_server_https_loopback_1MiB --steps 5 > $O/bench_c1.json 2> $O/bench_c1.err || { tail -20 $O/bench_c1.err; exit 1; }
for t in c2:c2_aes128gcm_64Ki_x_16KiB c3:c3_chacha20poly1305_64Ki_x_1.5KiB c4:c4_aes256gcm_1Mi_x_16KiB c5:c5_mixed_256Ki_x_64B-16KiB; do
  tag=${t%%:*}; cfg=${t#*:}
  bash tools/profile_round.sh $cfg r6_$tag || exit 1
  cp gpurun_out/prof_r6_$tag/run_kernel_stats.csv $O/${tag}_kernel_stats.csv
  python3 tools/kstats.py gpurun_out/prof_r6_$tag/run_kernel_trace.csv 3 > $O/${tag}_kernel_steady.json
  cp gpurun_out/prof_r6_${tag}_fetch/run_counter_collection.csv $O/${tag}_pmc_fetch.csv
  cp gpurun_out/prof_r6_${tag}_write/run_counter_collection.csv $O/${tag}_pmc_write.csv
  rm -rf gpurun_out/prof_r6_${tag}*
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_keysetup -o run --output-format csv -- python3 tools/key_setup_bench.py > $O/key_setup_bench.json 2> $O/key_setup_bench.err || exit 1
timeout -k 10 200 ./tools/single_call_floor > $O/single_call_floor.json 2>&1 || exit 1
ATLS_SINGLE_RESIDENT=1 timeout -k 10 200 ./tools/single_call_floor > $O/single_call_floor_resident.json 2>&1 || exit 1
cat $O/bench_default.json $O/single_call_floor.json $O/single_call_floor_resident.json
