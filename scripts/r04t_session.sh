#!/usr/bin/env bash
# GPU box, round 4 session t: final state — full GPU suite, smoke, default bench line
set -u
O=gpurun_out/r04t
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1" \
  "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1" \
  "timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err"
