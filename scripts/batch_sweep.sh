#!/usr/bin/env bash
# GPU box: bench lines over batch sizes, extra legs off, 10 warm-up steps
#   BATCHES="1 64 ..." bash scripts/batch_sweep.sh <tag>
set -u
TAG=${1:-sweep}
mkdir -p gpurun_out
for b in ${BATCHES:-1 64 256 512 768 1024 2048 4096}; do
  timeout -k 10 200 python bench.py --batch $b --steps 20 --warmup 10 --no-cpu-baseline --no-clock --no-ceiling \
      --extra-batches none --strong-batch 0 --parity-samples 16 > gpurun_out/${TAG}_$b.json 2>/dev/null || exit 3
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/${TAG}_$b.json') if l.startswith('{')][-1]
print('B=%-5d %9.0f /s  step %7.3f ms  br %7.3f ms  ks %.3f ms  parity %d/%d  ok=%s' % ($b, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['keyswitch_ms'], d['parity']['checked_per_rank'] - d['parity']['mismatches'], d['parity']['checked_per_rank'], d['truth_table_ok']))" | tee -a gpurun_out/${TAG}_summary.txt
done
