#!/usr/bin/env bash
# GPU box, round 4 session n: two ciphertexts per workgroup with the pair sync at the headline
# batches (TFHE_AMD_V6_PAIR=1) against the default one-ciphertext workgroups, alternating
set -u
O=gpurun_out/r04n
mkdir -p $O
bash scripts/gpu_session.sh \
  "BATCHES='1024 4096' timeout -k 10 300 bash scripts/batch_sweep.sh r04n/p0a > /dev/null 2>&1" \
  "TFHE_AMD_V6_PAIR=1 BATCHES='1024 4096' timeout -k 10 300 bash scripts/batch_sweep.sh r04n/p1a > /dev/null 2>&1" \
  "BATCHES='1024 4096' timeout -k 10 300 bash scripts/batch_sweep.sh r04n/p0b > /dev/null 2>&1" \
  "TFHE_AMD_V6_PAIR=1 BATCHES='1024 4096' timeout -k 10 300 bash scripts/batch_sweep.sh r04n/p1b > /dev/null 2>&1"
