cd $GRAFT_REPO_ROOT; export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 12288 24576 49152 65536 98304 131072 196608; do
  r=$(timeout -k 10 120 python bench.py --config c3_chacha20poly1305_64Ki_x_1.5KiB --records $n --no-cpu-baseline --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])") || exit 1
  echo "c3 records=$n: $r"
done
