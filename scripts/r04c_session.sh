#!/usr/bin/env bash
# GPU box, round 4 session c: host-pointer path (direct pageable DMA vs staging), LweSample batch,
# Tier-1 queue (released callers expected back), the tests that cover them
set -u
O=gpurun_out/r04c
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 400 python -u -m pytest tests/test_tier1.py tests/test_gpu_parity.py tests/test_multi_gpu.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/tests.txt 2>&1" \
  "timeout -k 10 200 python scripts/host_path_rate.py 1 64 1024 2048 4096 > $O/host_path_direct.jsonl 2>&1" \
  "TFHE_AMD_HOST_DIRECT=0 timeout -k 10 200 python scripts/host_path_rate.py 1 64 1024 2048 4096 > $O/host_path_staged.jsonl 2>&1" \
  "timeout -k 10 200 tests/callers/_bin/tier1_rate 16 1 8 64 > $O/tier1_rate.json 2>&1"
