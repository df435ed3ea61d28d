#!/bin/bash
# Round 6: the deferred last steps (gcm.hip ATLS_GCM_TAIL). Parity first (the new tail tests, the grouped and
# planned paths, C2 with a key per record against OpenSSL, whole C5 against the oracle), then same-box A/B by the
# engine switch ATLS_GCM_TAIL_ON=1/0: C2 with a key per record, C2, C5 whole, seal and open kernel ms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r6c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gcm_tail.py tests/test_gpu_gcm_groups.py tests/test_gpu_configs.py \
  tests/test_gpu_c5_full.py tests/test_gpu_parity.py tests/test_gpu_plan.py tests/test_wire_mode.py tests/test_gpu_c4_full.py \
  -x -v -m gpu --timeout 300 --timeout-method thread > $O/parity.txt 2>&1 || { tail -40 $O/parity.txt; exit 1; }
tail -1 $O/parity.txt
out=$O/ab_tail.log
: > $out
for round in 1 2 3; do
  for tok in c2_aes128gcm_64Ki_x_16KiB:0:65536 c2_aes128gcm_64Ki_x_16KiB c5_mixed_256Ki_x_64B-16KiB:262144 c4_aes256gcm_1Mi_x_16KiB; do
    IFS=: read -r cfg recs keys <<< "$tok"
    extra=""
    [ -n "${recs:-}" ] && [ "$recs" != 0 ] && extra="$extra --records $recs"
    [ -n "${keys:-}" ] && extra="$extra --key-slots $keys"
    for on in 1 0; do
      r=$(ATLS_GCM_TAIL_ON=$on timeout -k 10 150 python bench.py --config $cfg --no-cpu-baseline --no-configs --sustain-s 0 --steps 20 $extra 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); l=d['roofline'].get('lds') or {}; o=d['open']; print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], l.get('sclk_MHz'), l.get('frac'), o['kernel_ms'], o['frac'], o['plaintext_and_status_ok'])") || exit $?
      echo "round $round $tok tail_on=$on: GiBps seal_ms frac sclk lds_frac open_ms open_frac ok = $r" >> $out
    done
  done
done
cat $out
