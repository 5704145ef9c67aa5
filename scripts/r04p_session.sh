#!/usr/bin/env bash
# GPU box, round 4 session p: the full GPU suite and the smoke at the round's final state
set -u
O=gpurun_out/r04p
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1" \
  "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1" \
  "timeout -k 10 200 tests/callers/_bin/tier1_rate 32 1 8 64 > $O/tier1_rate.json 2>&1"
