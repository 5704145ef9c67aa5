#!/usr/bin/env bash
# blind-rotation kernel sweep over batch sizes (GPU box): scripts/br_sweep.sh "1 16 64" "4 5"
set -u
for b in $1; do
  for v in $2; do
    TFHE_AMD_BR=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch $b --no-cpu-baseline > gpurun_out/sw_${v}_${b}.log 2>&1
    rc=$?; [ $rc -ne 0 ] && exit $rc
    python3 - "$v" "$b" <<'PY'
import json, sys
v, b = sys.argv[1], sys.argv[2]
l = [x for x in open(f"gpurun_out/sw_{v}_{b}.log") if x.startswith("{")]
if not l:
    print(f"v{v} B={b}: no result"); sys.exit(0)
d = json.loads(l[-1])
print(f"v{v} B={b:>5} {d['value']:10.0f}/s  br {d['roofline']['kernel_ms']:8.3f} ms  ks {d['roofline']['keyswitch_ms']:.3f} ms ok={d['truth_table_ok']}")
PY
  done
done
