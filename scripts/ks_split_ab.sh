#!/usr/bin/env bash
set -u
mkdir -p gpurun_out
TFHE_AMD_KS_SPLIT=1000000 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_split.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_split.log; [ $rc -ne 0 ] && exit $rc
for b in 256 1024 4096; do
  for sp in 0 1000000 0 1000000; do
    TFHE_AMD_KS_SPLIT=$sp timeout -k 10 120 python bench.py --batch $b --no-cpu-baseline > gpurun_out/ksp_${b}_$sp.json 2>/dev/null || exit 3
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ksp_${b}_$sp.json') if l.startswith('{')][-1]
print('B=$b split<=$sp %.0f/s step %.3f ms br %.3f ks %.4f ms ok=%s' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['keyswitch_ms'], d['truth_table_ok']))"
  done
done
