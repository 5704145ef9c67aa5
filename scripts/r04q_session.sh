#!/usr/bin/env bash
# GPU box, round 4 session q: timing diagnostics (wrong results, guard off) pricing the radix-16
# forward for the next round: the forward A -> B transpose replaced by the permlane work a radix-16
# forward needs (permfwd), and both A <-> B transposes removed (notrab), against the same build
# unchanged, at B = 512 (paired kernel, pair sync) and 1024
set -u
mkdir -p gpurun_out/r04q
bash scripts/gpu_session.sh \
  "AB_BATCH=512 AB_STEPS=20 AB_WARMUP=10 AB_REPS=2 timeout -k 10 300 bash scripts/ab_bench.sh noguard permfwd-ng notrab-ng > gpurun_out/r04q/ab512.txt 2>&1" \
  "AB_BATCH=1024 AB_STEPS=20 AB_WARMUP=10 AB_REPS=2 timeout -k 10 300 bash scripts/ab_bench.sh noguard permfwd-ng notrab-ng > gpurun_out/r04q/ab1024.txt 2>&1"
