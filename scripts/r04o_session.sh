#!/usr/bin/env bash
# GPU box, round 4 session o: host-pointer batches above one round, pipelined slices (default)
# against one unsliced batch (TFHE_AMD_HOST_SLICE=0: every copy in first, the device batch's
# launches back to back, every copy out after), alternating
set -u
O=gpurun_out/r04o
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 200 python scripts/host_path_rate.py 2048 4096 > $O/sliced_a.jsonl 2>&1" \
  "TFHE_AMD_HOST_SLICE=0 timeout -k 10 200 python scripts/host_path_rate.py 2048 4096 > $O/unsliced_a.jsonl 2>&1" \
  "timeout -k 10 200 python scripts/host_path_rate.py 2048 4096 > $O/sliced_b.jsonl 2>&1" \
  "TFHE_AMD_HOST_SLICE=0 timeout -k 10 200 python scripts/host_path_rate.py 2048 4096 > $O/unsliced_b.jsonl 2>&1"
