#!/bin/bash
# C1 at scale after the double-buffered flush: stream parity tests, the loopback tool per phase, and the
# default bench line with the load settle (bench.py --load-settle-ms).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5c1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stream_native.py > $O/gpu_tests_stream.txt 2>&1 || { tail -30 $O/gpu_tests_stream.txt; exit 1; }
tail -1 $O/gpu_tests_stream.txt
for a in ${C1_RUNS:-"8 64 1" "8 64 8" "8 64 16" "16 64 8" "16 64 16" "2 256 8" "2 256 16" "4 256 8" "4 256 16"}; do
  timeout -k 10 120 tools/c1_loopback_native $a || exit 1
done > $O/c1_scale.log 2>&1
cat $O/c1_scale.log
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5c1/bench_default.json").read().strip().splitlines()[-1])
print(d["value"], d["roofline"]["frac"], d["roofline"]["lds"]["frac"], d["roofline"]["lds"]["sclk_MHz"], d["sustained"]["frac"])
for k, v in d["configs"].items():
    print(k, v["GiBps"], v["frac"], (v.get("lds") or {}).get("frac"))
PY
