#!/usr/bin/env bash
# GPU box, round 4 session m: the default bench line with the clock / ceiling runs after the legs
set -u
O=gpurun_out/r04m
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err" \
  "timeout -k 10 400 python bench.py > $O/bench_default2.json 2> $O/bench_default2.err"
