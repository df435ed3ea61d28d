#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline --sustain-s 0 > gpurun_out/b_open.json 2> gpurun_out/b_open.err || { tail -20 gpurun_out/b_open.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b_open.json").read().strip().splitlines()[-1])
print(d["value"], d["roofline"]["kernel_ms"], d["roofline"]["lds"]["frac"], d["roofline"]["lds"]["sclk_MHz"], d["open"])
for k, v in d["configs"].items():
    print(k, v["kernel_ms"], (v.get("lds") or {}).get("frac"), v["open"])
PY
