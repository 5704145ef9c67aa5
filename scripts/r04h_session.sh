#!/usr/bin/env bash
# GPU box, round 4 session h: host-side phases (TFHE_AMD_HOST_TRACE) of the record path under the
# Tier-1 queue and tfhe_amd_boots_batch, and a kernel + copy trace of the queue
set -u
O=gpurun_out/r04h
R=$(pwd)
mkdir -p $O
bash scripts/gpu_session.sh \
  "TFHE_AMD_HOST_TRACE=1 timeout -k 10 200 tests/callers/_bin/tier1_rate 8 64 > $O/tier1_rate.json 2> $O/tier1_trace.txt" \
  "TFHE_AMD_HOST_TRACE=1 timeout -k 10 300 python -u -m pytest tests/test_tier1.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k boots_batch > $O/boots_batch.txt 2>&1" \
  "cd /tmp && TMPDIR=/tmp timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/tr -o run -- $R/tests/callers/_bin/tier1_rate 8 64 > $R/$O/tier1_traced.json 2>&1"
bash scripts/gpu_session.sh \
  "timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err"
