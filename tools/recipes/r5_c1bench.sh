#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5c1b; mkdir -p $O
timeout -k 10 400 python -u bench.py --config c1_server_https_loopback_1MiB --steps 16 > $O/bench_c1.json 2> $O/bench_c1.err || { tail -20 $O/bench_c1.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c1.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['warmup'], d['python_StreamBatch'], d.get('native_phase_ms'), d['cpu_baseline']['value'])
for r in d['at_scale']['runs']: print(r.get('conns'), r.get('reps'), r.get('threads'), r.get('verified'), r.get('gpu_MBps'))"
