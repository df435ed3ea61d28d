#!/bin/bash
# Round 6: the product build (deferral compiled out, the planned ChaCha20-Poly1305 open reloading its key words):
# every GPU test, the smoke; C5 seal / open A/B of the key-word reload (variants base / kw0); the single-call
# floors through the resident server (latency unchanged by the launch holds); the clock probe's placement beside
# C2 and C4-whole seals; the default bench line. Outputs under gpurun_out/r6e/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r6e}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
O=$O PARITY=0 VARIANTS="base kw0" CONFIGS="c5_mixed_256Ki_x_64B-16KiB:262144 c5_mixed_256Ki_x_64B-16KiB" ROUNDS=3 \
  bash tools/recipes/r6_ab.sh kw || exit 1
for r in 1 2; do
  ATLS_SINGLE_RESIDENT=1 timeout -k 10 120 ./tools/single_call_floor > $O/floor_res_$r.json 2>&1 || { tail -5 $O/floor_res_$r.json; exit 1; }
  python3 -c "import json; d=json.load(open('$O/floor_res_$r.json')); print('resident round $r', {k: d[k] for k in ('chacha20poly1305_1537_seal_us','chacha20poly1305_1537_open_us','aes128gcm_1537_seal_us','aes128gcm_1537_open_us')})"
done
timeout -k 10 200 python -u tools/probe_overlap.py > $O/probe_overlap.jsonl 2>&1 || { tail -10 $O/probe_overlap.jsonl; exit 1; }
cat $O/probe_overlap.jsonl
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench_default.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['lds'].get('frac'),r['lds'].get('clock_in_window'),d['sustained'].get('lds_frac'))
for k,v in d['configs'].items(): print(k, v['GiBps'], v['kernel_ms'], v['frac'], v['open']['frac'], (v.get('lds') or {}).get('frac'), (v.get('lds') or {}).get('clock_in_window'))"
