#!/bin/bash
# Round 6 (third session): every GPU test and the smoke on the HEAD build (planned ChaCha20-Poly1305 open without
# scratch); C3's time split by ATLS_CHACHA_DBG timing builds (wrong results on purpose, no parity: 1 data keystream,
# 2 MAC, 4 full-block loads / stores; 3/5/6/7 their unions); C5 whole seal / open, the spill-free build against the
# round-start build; the default bench line. Outputs under gpurun_out/r6s3/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r6s3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
O=$O PARITY=0 VARIANTS="base dbg3 dbg4 dbg5 dbg6 dbg7" CONFIGS="c3_chacha20poly1305_64Ki_x_1.5KiB" ROUNDS=2 \
  bash tools/recipes/r6_ab.sh c3split || exit 1
O=$O PARITY=0 VARIANTS="base nospill" CONFIGS="c5_mixed_256Ki_x_64B-16KiB:262144" ROUNDS=3 \
  bash tools/recipes/r6_ab.sh c5spill || exit 1
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench_default.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['lds'].get('frac'),r['lds'].get('clock_in_window'),d['sustained'].get('lds_frac'))
for k,v in d['configs'].items(): print(k, v['GiBps'], v['kernel_ms'], v['frac'], v['open']['frac'], (v.get('lds') or {}).get('frac'))"
