#!/bin/bash
# Round 5: clock and power of the record kernels under sustained load (tools/clock_power.py), and the
# LDS-array PMC pass (SQ_LDS_IDX_ACTIVE, SQ_INSTS_LDS, GRBM_GUI_ACTIVE) of the C2 seal kernel and of the
# whole C4 batch (19-ms dispatches, where GRBM_GUI_ACTIVE / 8 / duration is the in-kernel clock within 3 %).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5clk; mkdir -p $O
timeout -k 10 300 python -u tools/clock_power.py --seconds 4 > $O/clock_power.json 2> $O/clock_power.err || { tail -30 $O/clock_power.err; exit 1; }
cat $O/clock_power.err
B="python3 bench.py --config c2_aes128gcm_64Ki_x_16KiB --steps 10 --warmup 3 --no-cpu-baseline --no-configs --sustain-s 0 --no-open"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/pmc_c2 -o run --output-format csv -- $B > $O/pmc_c2.log 2>&1 || { tail -20 $O/pmc_c2.log; exit 1; }
B4="python3 bench.py --config c4_aes256gcm_1Mi_x_16KiB --records 1048576 --steps 3 --warmup 1 --no-cpu-baseline --no-configs --sustain-s 0 --no-open"
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/pmc_c4w -o run --output-format csv -- $B4 > $O/pmc_c4w.log 2>&1 || { tail -20 $O/pmc_c4w.log; exit 1; }
python3 tools/pmc_summary.py $(ls $O/pmc_c2/*/run_counter_collection.csv 2>/dev/null || ls $O/pmc_c2/run_counter_collection.csv) gcm_kernel 3 > $O/pmc_c2_summary.json
python3 tools/pmc_summary.py $(ls $O/pmc_c4w/*/run_counter_collection.csv 2>/dev/null || ls $O/pmc_c4w/run_counter_collection.csv) gcm_kernel 1 > $O/pmc_c4w_summary.json
cat $O/pmc_c2_summary.json $O/pmc_c4w_summary.json
tail -3 $O/pmc_c2.log
