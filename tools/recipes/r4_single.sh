#!/bin/bash
# Round 4: the Cipher-trait single call -- launch floors (empty kernels, a 3.7 KB argument block), the
# phase clocks of the ChaCha20-Poly1305 single-call kernel (timing build), and the product's latencies.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 120 ./tools/single_call_floor > gpurun_out/r4/single_call_floor.json 2>&1 || exit 1
cat gpurun_out/r4/single_call_floor.json
ATLS_LIB=$PWD/anothertls_amd/variants/libatls_latstamps.so timeout -k 10 180 python3 tools/single_call_stamps.py > gpurun_out/r4/single_call_stamps.json 2>&1 || { cat gpurun_out/r4/single_call_stamps.json; exit 1; }
cat gpurun_out/r4/single_call_stamps.json
