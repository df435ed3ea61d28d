#!/bin/bash
# Round 4: synchronous engine returns through a completion flag (engine.cpp finish) -- every GPU test, the
# smoke, the single-call floors (one-key install with a stream sync and with atls_engine_sync), the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
export ATLS_SYNC_FLAG=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 120 ./tools/single_call_floor > $O/single_call_floor.json 2>&1 || { cat $O/single_call_floor.json; exit 1; }
cat $O/single_call_floor.json
timeout -k 10 300 python3 tools/key_setup_bench.py > $O/key_setup_bench.json 2>&1 || { cat $O/key_setup_bench.json; exit 1; }
cat $O/key_setup_bench.json
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -c 600 $O/bench_default.json
