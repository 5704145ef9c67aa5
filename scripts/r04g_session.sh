#!/usr/bin/env bash
# GPU box, round 4 session g: Tier-1 queue (record path, tree wake-up, device variance with the
# uniform-row table), host-pointer path phases (TFHE_AMD_HOST_TRACE), LweSample batches
set -u
O=gpurun_out/r04g
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 400 python -u -m pytest tests/test_tier1.py tests/test_gpu_parity.py tests/test_l1_exports.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/tests.txt 2>&1" \
  "timeout -k 10 200 tests/callers/_bin/tier1_rate 16 1 8 64 > $O/tier1_rate.json 2>&1" \
  "timeout -k 10 200 tests/callers/_bin/tier1_rate 32 64 > $O/tier1_rate_32.json 2>&1" \
  "timeout -k 10 200 python scripts/host_path_rate.py 1 64 1024 2048 4096 > $O/host_path.jsonl 2>&1" \
  "TFHE_AMD_HOST_TRACE=1 timeout -k 10 200 python scripts/host_path_rate.py 1024 4096 > $O/host_path_trace.jsonl 2> $O/host_trace.txt"
