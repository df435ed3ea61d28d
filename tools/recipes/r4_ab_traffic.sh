#!/bin/bash
# Round 4: FETCH_SIZE / WRITE_SIZE of one config's dominant kernel per library variant (separate --pmc
# passes, MI355X_MICROARCH.md §HBM), reduced by tools/ab_traffic.py.
# Usage: VARIANTS="base c3stage" bash tools/recipes/r4_ab_traffic.sh <tag> <config> <kernel substring> <alg bytes>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag=$1; cfg=$2; kern=$3; alg=$4
d=gpurun_out/r4/tr_$tag
mkdir -p $d
for v in ${VARIANTS:-base}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    s=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    ATLS_LIB=$PWD/anothertls_amd/variants/libatls_$v.so timeout -s KILL 120 rocprofv3 --pmc $c -d $d/${v}_$s -o run --output-format csv -- python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-configs --no-open > $d/${v}_$s.log 2>&1 || { tail -5 $d/${v}_$s.log; exit 1; }
  done
done
python3 tools/ab_traffic.py $d "$kern" $alg ${VARIANTS:-base} | tee gpurun_out/r4/ab_${tag}_traffic.json
