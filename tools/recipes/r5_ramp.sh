#!/bin/bash
# Ramped host-pipeline chunks: parity (host pipeline + stream tests), then PCIe-inclusive C2, the socket-path
# batch probe and C1 at scale, ramp on (default) against flat chunks (ATLS_CHUNK_FIRST_MB=0), 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5ramp; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_host_pipeline.py tests/test_gpu_stream_native.py > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
for r in 1 2; do
for f in 4 0; do
  ATLS_CHUNK_FIRST_MB=$f timeout -k 10 200 python -u bench.py --pcie --no-configs --no-cpu-baseline --sustain-s 0 --no-open --steps 5 --load-settle-ms 0 > $O/pcie_$f.json 2> $O/pcie_$f.err || { tail -5 $O/pcie_$f.err; exit 1; }
  python - $f $r <<'PY'
import json, sys
f = sys.argv[1]
d = json.loads(open(f"gpurun_out/r5ramp/pcie_{f}.json").read().strip().splitlines()[-1])
print("round", sys.argv[2], "first_MB", f, {k: v for k, v in d.items() if k.startswith("pcie")}, flush=True)
PY
  ATLS_CHUNK_FIRST_MB=$f timeout -k 10 200 python -u tools/host_batch_probe.py 2>/dev/null | sed "s/^/round $r first_MB $f /"
  for a in "16 64 8" "4 256 8"; do
    ATLS_CHUNK_FIRST_MB=$f timeout -k 10 120 tools/c1_loopback_native $a | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('round $r first_MB $f c1', d['conns'], d['reps'], d['threads'], d['verified'], d['gpu_MBps'], d['phase_ms'])"
  done
done
done
