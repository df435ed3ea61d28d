#!/bin/bash
# Same-box A/B of anothertls_amd/variants/libatls_*.so on C3 with HBM traffic: parity, one FETCH_SIZE and
# one WRITE_SIZE pass per variant (seal and open kernels, KiB per dispatch; FETCH doubled as in
# tools/traffic.py), then tools/recipes/sessions/_ab_c3.sh's 3 timing rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
B="python3 bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --steps 5 --warmup 2 --no-cpu-baseline"
for lib in anothertls_amd/variants/libatls_*.so; do
  n=$(basename $lib .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    ATLS_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/tr_${n}_$c -o run --output-format csv -- $B > gpurun_out/tr_${n}_$c.log 2>&1 || { echo "pmc $n $c rc=$?"; exit 1; }
  done
  python3 - "$n" <<'PY'
import csv, glob, sys, collections
n = sys.argv[1]
alg = 65536 * (2 * 1537 + 16)
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/tr_{n}_{c}/**/run_counter_collection.csv", recursive=True)[0]
    v = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == c and "chacha_kernel" in r["Kernel_Name"]:
            v[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]) * 1024 * (2 if c == "FETCH_SIZE" else 1))
    for k, xs in v.items():
        xs = xs[2:] or xs
        out.setdefault(k, {})[c] = sum(xs) / len(xs)
for k, d in out.items():
    t = d.get("FETCH_SIZE", 0) + d.get("WRITE_SIZE", 0)
    print(f"{n} {k}: fetch {d.get('FETCH_SIZE', 0)/1e6:.1f} MB write {d.get('WRITE_SIZE', 0)/1e6:.1f} MB traffic/alg {t/alg:.3f}")
PY
done
bash tools/recipes/sessions/_ab_c3.sh
