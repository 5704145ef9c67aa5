#!/usr/bin/env bash
# GPU box, round 4 session r: issue-priority policies on this round's kernel at B = 1024 and 512
# (policy:shift; 5:3 is the default for one-round launches), two passes
set -u
mkdir -p gpurun_out/r04r
bash scripts/gpu_session.sh \
  "PS_WARMUP=10 timeout -k 10 400 bash scripts/prio_sweep.sh 1024 '5:3 0:3 5:2 5:4 2:3 5:3 0:3 5:2 5:4' > gpurun_out/r04r/p1024.txt 2>&1" \
  "PS_WARMUP=10 timeout -k 10 300 bash scripts/prio_sweep.sh 512 '5:3 0:3 5:2 5:4 5:3 0:3' > gpurun_out/r04r/p512.txt 2>&1"
