#!/usr/bin/env bash
# GPU box, round 4 session y: the binding reading int32 arrays in place (no per-call copies):
# full GPU suite, host-pointer rate against the synchronous device path, default bench line
set -u
O=gpurun_out/r04y
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1" \
  "timeout -k 10 200 python scripts/host_path_rate.py 64 1024 2048 4096 > $O/host_path.jsonl 2>&1" \
  "TFHE_AMD_HOST_TRACE=1 timeout -k 10 200 python scripts/host_path_rate.py 1024 4096 > $O/host_path_trace.jsonl 2> $O/host_trace.txt" \
  "timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err"
