#!/usr/bin/env bash
# GPU box: small-batch key switch, fully unrolled vs unroll 4, per batch (TFHE_AMD_KS_UNROLL)
set -u
mkdir -p gpurun_out
for b in ${BATCHES:-1 2 4 8 16 32 64}; do
  for u in 0 96; do
    TFHE_AMD_KS_UNROLL=$u timeout -k 10 120 python bench.py --steps 10 --warmup 2 --batch $b --no-cpu-baseline > gpurun_out/ku_${b}_$u.json 2>&1 || exit 3
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ku_${b}_$u.json') if l.startswith('{')][-1]
print('B=$b unroll_max=$u ks %.4f ms br %.3f ok=%s' % (d['roofline']['keyswitch_ms'], d['roofline']['kernel_ms'], d['truth_table_ok']))"
  done
done
