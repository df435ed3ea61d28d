#!/bin/bash
# SQ PMC pass (LDS / VALU activity) over C2 for one library: bash tools/pmc_lds_one.sh <lib> <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="python3 bench.py --config c2_aes128gcm_64Ki_x_16KiB --steps 5 --warmup 2 --no-cpu-baseline"
ATLS_LIB=$PWD/$1 timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_lds_$2 -o run --output-format csv -- $B > gpurun_out/pmc_lds_$2.log 2>&1
