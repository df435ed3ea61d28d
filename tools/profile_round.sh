#!/bin/bash
# rocprofv3 evidence for the bench configs: kernel-trace stats, then FETCH_SIZE / WRITE_SIZE in
# separate --pmc passes (MI355X_MICROARCH.md §HBM), each pass under its own time limit.
# Usage: bash tools/profile_round.sh <config> <tag>   (outputs under gpurun_out/prof_<tag>*)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
cfg=$1; tag=$2; extra=${3:-}
B="python3 bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-configs --sustain-s 0 $extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- $B > gpurun_out/prof_$tag.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_${tag}_fetch -o run --output-format csv -- $B > gpurun_out/prof_${tag}_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_${tag}_write -o run --output-format csv -- $B > gpurun_out/prof_${tag}_write.log 2>&1 || exit $?
echo "profiled $cfg"
