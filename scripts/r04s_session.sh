#!/usr/bin/env bash
# GPU box, round 4 session s: paired launches without an issue-priority policy (parity, B = 512)
set -u
O=gpurun_out/r04s
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k 'paired or gate_batch or mux' > $O/tests.txt 2>&1" \
  "BATCHES='512 384' timeout -k 10 300 bash scripts/batch_sweep.sh r04s/a > /dev/null 2>&1" \
  "BATCHES='512' timeout -k 10 300 bash scripts/batch_sweep.sh r04s/b > /dev/null 2>&1"
