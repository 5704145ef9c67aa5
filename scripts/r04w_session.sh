#!/usr/bin/env bash
# GPU box, round 4 session w: the one-ciphertext kernel's pair sync at the latency-class batches
# (B = 1, 64, 256: one workgroup per CU at most), alternating with the default
set -u
mkdir -p gpurun_out/r04w
bash scripts/gpu_session.sh \
  "BATCHES='1 64 256' timeout -k 10 300 bash scripts/batch_sweep.sh r04w/ps0a > /dev/null 2>&1" \
  "TFHE_AMD_V6_PAIRSYNC=1 BATCHES='1 64 256' timeout -k 10 300 bash scripts/batch_sweep.sh r04w/ps1a > /dev/null 2>&1" \
  "BATCHES='1 64 256' timeout -k 10 300 bash scripts/batch_sweep.sh r04w/ps0b > /dev/null 2>&1" \
  "TFHE_AMD_V6_PAIRSYNC=1 BATCHES='1 64 256' timeout -k 10 300 bash scripts/batch_sweep.sh r04w/ps1b > /dev/null 2>&1"
