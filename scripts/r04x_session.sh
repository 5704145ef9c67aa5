#!/usr/bin/env bash
# GPU box, round 4 session x: host-pointer path against the device path called synchronously
set -u
mkdir -p gpurun_out/r04x
bash scripts/gpu_session.sh \
  "timeout -k 10 200 python scripts/host_path_rate.py 64 1024 4096 > gpurun_out/r04x/host_path.jsonl 2>&1" \
  "timeout -k 10 200 python scripts/host_path_rate.py 64 1024 4096 > gpurun_out/r04x/host_path2.jsonl 2>&1"
