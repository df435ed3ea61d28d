#!/bin/bash
# Same-box timing of the shared-GHASH-table experiment (ATLS_DBG_SHARED_GHASH, wrong tags):
# base 12 waves vs one table per workgroup at 12 and 16 waves, C2 and C4, interleaved, 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {  # label lib waves cfg
  r=$(ATLS_LIB=$PWD/$2 ATLS_GCM_WAVES=$3 timeout -k 10 120 python bench.py --config $4 --no-cpu-baseline --steps 10 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])") || exit $?
  echo "$4 $1: $r"
}
for round in 1 2; do
  for cfg in c2_aes128gcm_64Ki_x_16KiB c4_aes256gcm_1Mi_x_16KiB; do
    run base12 anothertls_amd/libatls.so 12 $cfg || exit $?
    run shared12 anothertls_amd/variants/libatls_shared.so 12 $cfg || exit $?
    run shared16 anothertls_amd/variants/libatls_shared.so 16 $cfg || exit $?
  done
done
