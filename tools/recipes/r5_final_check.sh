#!/bin/bash
# The round-end check as the driver runs it: every GPU test, the smoke, bench.py --gpus 1 --steps 20 --warmup 5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5fc; mkdir -p $O
O=$O bash tools/recipes/r5_full_tests.sh || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['lds']['frac'], r['lds']['sclk_MHz'], d['open']['frac'], d['open'].get('lds'), d['sustained']['frac'])
for k,v in d['configs'].items(): print(k, v['GiBps'], v['frac'], (v.get('lds') or {}).get('frac'), v['open']['frac'])"
