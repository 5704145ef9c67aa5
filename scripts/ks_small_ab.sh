#!/usr/bin/env bash
set -u
mkdir -p gpurun_out
for b in 1 4 16 32 64 128; do
  for th in 0 1000; do
    TFHE_AMD_KS_SMALL=$th timeout -k 10 120 python bench.py --batch $b --no-cpu-baseline > gpurun_out/kss_${b}_$th.json 2>/dev/null || exit 3
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/kss_${b}_$th.json') if l.startswith('{')][-1]
print('B=$b small<=$th %.0f/s step %.3f ms br %.3f ks %.4f ms ok=%s' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['keyswitch_ms'], d['truth_table_ok']))"
  done
done
