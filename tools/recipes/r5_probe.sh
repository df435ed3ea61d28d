#!/bin/bash
# Round 5, first pass: what the box offers for clock / power readings, the GPU tests (C5 whole batch
# included) and the default bench line (roofline.lds, C5 whole).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5a; mkdir -p $O
( which amd-smi rocm-smi; for c in /sys/class/drm/card*/device; do echo "== $c"; ls $c/hwmon/*/ 2>/dev/null; cat $c/hwmon/*/freq1_input $c/hwmon/*/power1_average $c/hwmon/*/power1_input $c/hwmon/*/power1_cap 2>/dev/null; cat $c/pp_dpm_sclk 2>/dev/null; done ) > $O/sysfs.txt 2>&1
timeout -k 5 60 amd-smi metric --help > $O/amdsmi_help.txt 2>&1
timeout -k 5 60 amd-smi metric -p -c --json > $O/amdsmi_metric.json 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -30 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
