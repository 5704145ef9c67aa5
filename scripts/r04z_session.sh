#!/usr/bin/env bash
# GPU box, round 4 session z: one-round host batches staged in four chunks from 1 024 gates (copy
# pool from 512 KB): parity of the host paths, host-pointer rate, Tier-1 queue, bench line
set -u
O=gpurun_out/r04z
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_tier1.py tests/test_multi_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1" \
  "timeout -k 10 200 python scripts/host_path_rate.py 64 1024 2048 4096 > $O/host_path.jsonl 2>&1" \
  "timeout -k 10 200 python scripts/host_path_rate.py 1024 > $O/host_path2.jsonl 2>&1" \
  "timeout -k 10 200 tests/callers/_bin/tier1_rate 32 64 > $O/tier1_rate.json 2>&1" \
  "timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err"
