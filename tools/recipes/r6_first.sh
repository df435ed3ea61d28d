#!/bin/bash
# Round 6, first GPU pass: every GPU test (new: resident calls beside batches, interleaved socket writes and peer
# close, C2 with a key per record against OpenSSL), the smoke, the default bench line (lds.frac now from the timed
# launches' own clock), the LDS gather microbenchmark (plain and under SQ_LDS_IDX_ACTIVE), and two wave-state PMC
# passes of the C2 seal kernel (VERDICT r5 #2's counter list). Outputs under gpurun_out/r6a/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r6a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 120 ./tools/ubench/lds_gather_ubench > $O/lds_gather.jsonl 2>&1 || { tail -20 $O/lds_gather.jsonl; exit 1; }
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
have() { for c in "$@"; do grep -qw "$c" $O/counters.txt && printf '%s ' "$c"; done; }
U=$(have SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU)
echo "ubench pass: $U"
timeout -s KILL 120 rocprofv3 --pmc $U GRBM_GUI_ACTIVE -d $O/ub -o run --output-format csv -- ./tools/ubench/lds_gather_ubench > $O/ub.log 2>&1 || exit $?
A=$(have SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS)
B=$(have SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM)
echo "pass a: $A"; echo "pass b: $B"
CMD="python3 bench.py --config c2_aes128gcm_64Ki_x_16KiB --steps 5 --warmup 2 --no-cpu-baseline --no-configs --sustain-s 0 --load-settle-ms 300 --no-open"
timeout -s KILL 150 rocprofv3 --pmc $A GRBM_GUI_ACTIVE -d $O/a -o run --output-format csv -- $CMD > $O/a.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc $B GRBM_GUI_ACTIVE -d $O/b -o run --output-format csv -- $CMD > $O/b.log 2>&1 || exit $?
for p in a b; do
  f=$(ls $O/$p/*/run_counter_collection.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls $O/$p/run_counter_collection.csv)
  python3 tools/pmc_summary.py $f gcm_kernel 2 > $O/summary_$p.json
  cat $O/summary_$p.json
done
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'],d['roofline']['frac'],d['roofline']['lds'],d.get('sustained'))"
