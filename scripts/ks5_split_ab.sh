#!/usr/bin/env bash
# GPU box: key-switch time of ks-v5 by key-index split (TFHE_AMD_KS5_SPLIT) and batch (dev tool)
set -u
for B in ${KS_BATCHES:-128 256 512 1024 4096}; do
for sp in ${KS_SPLITS:-1 2 4 8}; do
  TFHE_AMD_KS5_SPLIT=$sp timeout -k 10 200 python bench.py --steps 10 --warmup 2 --batch $B --no-cpu-baseline --no-clock --no-ceiling --extra-batches '' --strong-batch 0 > gpurun_out/kssp_${B}_$sp.json 2>&1 || exit 1
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/kssp_${B}_$sp.json') if l.startswith('{')][-1]
print('B=$B split=$sp  %.0f /s  br %.3f ks %.3f ms ok=%s' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['keyswitch_ms'], d['truth_table_ok']))"
done; done
