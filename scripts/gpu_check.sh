#!/usr/bin/env bash
# GPU box: parity suite, then bench lines at B = 1024 / 4096 / 1 for the given kernel generations
#   bash scripts/gpu_check.sh "0 7"
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for b in ${BATCHES:-1024 4096 1}; do
  for v in ${1:-0}; do
    TFHE_AMD_BR=$v timeout -k 10 120 python bench.py --steps 5 --warmup 1 --batch $b --no-cpu-baseline > gpurun_out/chk_v${v}_$b.json 2>&1 || exit 3
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/chk_v${v}_$b.json') if l.startswith('{')][-1]
print('br=$v B=$b %.0f/s br %.3f ms ks %.3f ok=%s %s' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['keyswitch_ms'], d['truth_table_ok'], d['engine']))"
  done
done
