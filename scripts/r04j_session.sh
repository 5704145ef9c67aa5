#!/usr/bin/env bash
# GPU box, round 4 session j: the paired kernel's waves meeting through LDS counters instead of the
# workgroup barrier (TFHE_AMD_V6P_PAIRSYNC=1: parity, A/B at B = 512 / 384), then the round-end set
# — full GPU suite, smoke, default bench line, rocprofv3 kernel trace/stats + PMC passes
set -u
O=gpurun_out/r04j
mkdir -p $O
bash scripts/gpu_session.sh \
  "TFHE_AMD_V6P_PAIRSYNC=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k 'paired or gate_batch or mux or woks or guard' > $O/tests_pairsync.txt 2>&1" \
  "BATCHES='512 384' timeout -k 10 300 bash scripts/batch_sweep.sh r04j/ps0 > /dev/null 2>&1" \
  "TFHE_AMD_V6P_PAIRSYNC=1 BATCHES='512 384' timeout -k 10 300 bash scripts/batch_sweep.sh r04j/ps1 > /dev/null 2>&1" \
  "timeout -k 10 200 tests/callers/_bin/tier1_rate 32 1 8 64 > $O/tier1_rate.json 2>&1" \
  "timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1" \
  "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1" \
  "timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err"
