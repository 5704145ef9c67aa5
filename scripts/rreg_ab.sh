#!/usr/bin/env bash
# the small-batch launches' rotation form: LDS extension (default at B <= CUs) vs TFHE_AMD_V6_RREG=1
# (the register rotation, its scalar-branch permutation form); RREG_BATCHES (default "1 256")
set -u
mkdir -p gpurun_out
for rep in 1 2 3; do
for v in 0 1; do
  for b in ${RREG_BATCHES:-1 256}; do
    TFHE_AMD_V6_RREG=$v timeout -k 10 200 python bench.py --batch $b --steps 40 --warmup 10 --no-cpu-baseline --no-clock --no-ceiling --no-circuits --extra-batches none --strong-batch none --host-batches none --parity-samples 8 > gpurun_out/rreg_${v}_${b}_$rep.json 2>/dev/null || exit 3
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/rreg_${v}_${b}_$rep.json') if l.startswith('{')][-1]
print('RREG=$v B=$b rep $rep  %8.1f /s  br %.4f ms  parity %d/%d' % (d['value'], d['roofline']['kernel_ms'], d['parity']['checked_per_rank']-d['parity']['mismatches'], d['parity']['checked_per_rank']))" | tee -a gpurun_out/rreg_ab.txt
  done
done
done
