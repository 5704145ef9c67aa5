#!/usr/bin/env bash
# GPU box: default bench line (with CPU baseline) + batch sweep for DESIGN.md §5.3
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 3
for b in ${BATCHES:-1 64 256 1024 2048 4096}; do
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline > gpurun_out/bt_$b.json 2>/dev/null || exit 3
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/bt_$b.json') if l.startswith('{')][-1]
print('B=$b %.0f/s step %.3f ms br %.3f ms ks %.3f ok=%s' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['keyswitch_ms'], d['truth_table_ok']))" | tee -a gpurun_out/bt_summary.txt
done
