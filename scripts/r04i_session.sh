#!/usr/bin/env bash
# GPU box, round 4 session i: Tier-1 queue policies (merge with a 200 us window floor vs overlap)
set -u
O=gpurun_out/r04i
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 200 tests/callers/_bin/tier1_rate 16 1 8 64 > $O/tier1_merge.json 2>&1" \
  "TFHE_AMD_TIER1_MERGE=0 timeout -k 10 200 tests/callers/_bin/tier1_rate 16 1 8 64 > $O/tier1_nomerge.json 2>&1" \
  "timeout -k 10 200 tests/callers/_bin/tier1_rate 32 64 > $O/tier1_merge_32.json 2>&1" \
  "TFHE_AMD_TIER1_MERGE=0 timeout -k 10 200 tests/callers/_bin/tier1_rate 32 64 > $O/tier1_nomerge_32.json 2>&1" \
  "timeout -k 10 200 tests/callers/_bin/tier1_rate 4 256 > $O/tier1_merge_256.json 2>&1" \
  "TFHE_AMD_TIER1_MERGE=0 timeout -k 10 200 tests/callers/_bin/tier1_rate 4 256 > $O/tier1_nomerge_256.json 2>&1" \
  "timeout -k 10 300 python -u -m pytest tests/test_tier1.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/tests.txt 2>&1"
