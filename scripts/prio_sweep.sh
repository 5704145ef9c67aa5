#!/usr/bin/env bash
# issue-priority policy sweep (GPU box): scripts/prio_sweep.sh <batch> "<policy:shift> ..."
set -u
mkdir -p gpurun_out
for ps in $2; do
  p=${ps%%:*}; sft=${ps#*:}
  TFHE_AMD_PRIO=$p TFHE_AMD_PRIO_S=$sft timeout -k 10 120 python bench.py --steps 10 --warmup ${PS_WARMUP:-2} --batch $1 --no-cpu-baseline --no-clock --no-ceiling --extra-batches none --strong-batch 0 > gpurun_out/ps_${1}_${p}_${sft}.json 2>&1 || exit 3
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ps_${1}_${p}_${sft}.json') if l.startswith('{')][-1]
print('B=$1 policy $p shift $sft: %.0f/s br %.3f ms ok=%s' % (d['value'], d['roofline']['kernel_ms'], d['truth_table_ok']))" | tee -a gpurun_out/ps_summary.txt
done
