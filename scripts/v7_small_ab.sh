#!/usr/bin/env bash
set -u
mkdir -p gpurun_out
TFHE_AMD_BR=7 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_v7.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_v7.log; [ $rc -ne 0 ] && exit $rc
for b in 1 16 64 256 512; do
  for v in 0 7; do
    TFHE_AMD_BR=$v timeout -k 10 120 python bench.py --batch $b --no-cpu-baseline > gpurun_out/v7s_${b}_$v.json 2>/dev/null || exit 3
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/v7s_${b}_$v.json') if l.startswith('{')][-1]
print('B=$b br=$v %.0f/s step %.3f ms br %.3f ms ok=%s' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['truth_table_ok']))"
  done
done
