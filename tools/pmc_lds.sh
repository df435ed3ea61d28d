#!/bin/bash
# One SQ PMC pass (LDS / VALU activity) over C2 for the base kernel and the shared-GHASH 16-wave
# timing build (ATLS_DBG_SHARED_GHASH). Outputs under gpurun_out/pmc_lds_<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="python3 bench.py --config c2_aes128gcm_64Ki_x_16KiB --steps 5 --warmup 2 --no-cpu-baseline"
ATLS_LIB=$PWD/anothertls_amd/libatls.so ATLS_GCM_WAVES=12 timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_lds_base12 -o run --output-format csv -- $B > gpurun_out/pmc_lds_base12.log 2>&1 || exit $?
ATLS_LIB=$PWD/anothertls_amd/variants/libatls_shared.so ATLS_GCM_WAVES=16 timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_lds_shared16 -o run --output-format csv -- $B > gpurun_out/pmc_lds_shared16.log 2>&1 || exit $?
echo done
