#!/usr/bin/env bash
# GPU box, round 4 final check of the committed build: GPU suite and smoke
set -u
O=gpurun_out/r04zz
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1" \
  "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1"
