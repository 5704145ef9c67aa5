#!/usr/bin/env bash
# GPU box, round 4 session l: the paired kernel with the pair sync (default) against the barrier
# (TFHE_AMD_V6P_PAIRSYNC=0) at B = 512 on one box, twice each, then the default bench line
set -u
O=gpurun_out/r04l
mkdir -p $O
bash scripts/gpu_session.sh \
  "BATCHES='512' timeout -k 10 300 bash scripts/batch_sweep.sh r04l/ps1a > /dev/null 2>&1" \
  "TFHE_AMD_V6P_PAIRSYNC=0 BATCHES='512' timeout -k 10 300 bash scripts/batch_sweep.sh r04l/ps0a > /dev/null 2>&1" \
  "BATCHES='512' timeout -k 10 300 bash scripts/batch_sweep.sh r04l/ps1b > /dev/null 2>&1" \
  "TFHE_AMD_V6P_PAIRSYNC=0 BATCHES='512' timeout -k 10 300 bash scripts/batch_sweep.sh r04l/ps0b > /dev/null 2>&1" \
  "timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err"
