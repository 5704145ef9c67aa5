#!/usr/bin/env bash
# GPU box, round 4 session u: the default bench line with 0.3 s of warm-up per leg, twice, and the
# B = 512 batch in isolation for comparison
set -u
O=gpurun_out/r04u
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err" \
  "BATCHES='512' timeout -k 10 300 bash scripts/batch_sweep.sh r04u/iso > /dev/null 2>&1" \
  "timeout -k 10 400 python bench.py > $O/bench_default2.json 2> $O/bench_default2.err"
