#!/bin/bash
# C2's fixed cost per launch: the same records (16 per key) at 1/4x .. 4x C2's count, kernel ms per record
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5sw; mkdir -p $O
for n in 16384 32768 65536 131072 262144; do
  timeout -k 10 200 python -u bench.py --records $n --key-slots $((n / 16)) --no-configs --no-cpu-baseline --sustain-s 0 --no-open --steps 20 > $O/sweep_$n.json 2> $O/sweep_$n.err || { tail -5 $O/sweep_$n.err; exit 1; }
  python - $n <<'PY'
import json, sys
n = int(sys.argv[1])
d = json.loads(open(f"gpurun_out/r5sw/sweep_{n}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(n, r["kernel_ms"], round(r["kernel_ms"] / n * 65536, 4), r["frac"], r["lds"]["frac"], r["lds"]["sclk_MHz"], flush=True)
PY
done
