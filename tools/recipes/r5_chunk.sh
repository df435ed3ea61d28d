#!/bin/bash
# PCIe-inclusive C2 (host batches) against the engine's chunk size (ATLS_CHUNK_MB), 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5ch; mkdir -p $O
for r in 1 2; do
for mb in 16 32 64 128 256; do
  ATLS_CHUNK_MB=$mb timeout -k 10 200 python -u bench.py --pcie --no-configs --no-cpu-baseline --sustain-s 0 --no-open --steps 5 --load-settle-ms 0 > $O/chunk_$mb.json 2> $O/chunk_$mb.err || { tail -5 $O/chunk_$mb.err; exit 1; }
  python - $mb $r <<'PY'
import json, sys
mb = sys.argv[1]
d = json.loads(open(f"gpurun_out/r5ch/chunk_{mb}.json").read().strip().splitlines()[-1])
print("round", sys.argv[2], "chunk_MB", mb, {k: v for k, v in d.items() if k.startswith("pcie")}, flush=True)
PY
done
done
