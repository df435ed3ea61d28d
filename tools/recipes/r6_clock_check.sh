#!/bin/bash
# Round 6 (VERDICT r5 #1's check): on one box, the default bench line's C2 roofline.lds (clock probe beside the
# timed launches) and its sustained leg, then the in-kernel clock stamps of the diagnostic build (every wave's
# s_memtime / s_memrealtime over the kernel body, tools/clock_check.py) -- the three LDS-array fractions of the same tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r6clk}; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-configs --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
ATLS_LIB=$PWD/anothertls_amd/variants/libatls_clk.so timeout -k 10 300 python -u tools/clock_check.py --seconds 2 --configs c2,c4 > $O/clock_check.json 2> $O/clock_check.err || { tail -30 $O/clock_check.err; exit 1; }
cat $O/clock_check.err
python3 -c "
import json
d=json.load(open('$O/bench_c2.json')); r=d['roofline']['lds']; s=d['sustained']
print('bench window', r['frac'], r['sclk_MHz'], r['kernel_ms'], '| sustained', s['lds_frac'], s['sclk_MHz'], s['kernel_ms'])
c=json.load(open('$O/clock_check.json'))
for x in c['runs']:
    cyc = 414076928 if 'c2' in x['config'] else 1097113600
    print(x['config'], 'in-kernel', round(cyc / (256 * x['in_kernel_MHz'] * 1e3 * x['kernel_ms']), 4), x['in_kernel_MHz'], x['kernel_ms'], 'probe', x['probe_MHz_median'])
"
