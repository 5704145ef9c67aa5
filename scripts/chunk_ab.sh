#!/usr/bin/env bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for b in 1024 2048 4096 3000; do
  for ch in default 0; do
    if [ $ch = default ]; then unset TFHE_AMD_CHUNK; else export TFHE_AMD_CHUNK=$ch; fi
    timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline > gpurun_out/ch_${b}_$ch.json 2>/dev/null || exit 3
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ch_${b}_$ch.json') if l.startswith('{')][-1]
print('B=$b chunk=$ch %.0f/s step %.3f ms br %.3f ms ks %.3f ok=%s' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['keyswitch_ms'], d['truth_table_ok']))"
  done
done
