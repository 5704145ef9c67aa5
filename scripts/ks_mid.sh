#!/usr/bin/env bash
set -u
mkdir -p gpurun_out
for b in 128 512 768; do
  for sp in 0 1000000; do
    TFHE_AMD_KS_SPLIT=$sp timeout -k 10 120 python bench.py --batch $b --no-cpu-baseline > gpurun_out/ksm_${b}_$sp.json 2>/dev/null || exit 3
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ksm_${b}_$sp.json') if l.startswith('{')][-1]
print('B=$b split<=$sp %.0f/s step %.3f ms br %.3f ks %.4f ms ok=%s' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['keyswitch_ms'], d['truth_table_ok']))"
  done
done
