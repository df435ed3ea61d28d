#!/bin/bash
# Kernel time of library variants (anothertls_amd/variants/*.so matching $1): bench.py per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in anothertls_amd/variants/$1; do
  r=$(ATLS_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 ${@:2} 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])") || exit $?
  echo "$(basename $lib): $r"
done
