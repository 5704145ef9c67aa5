#!/usr/bin/env bash
# GPU box, round 4 session k: the pair-synced paired kernel as the default (parity incl. the barrier
# variant, smoke, default bench line with its B = 512 leg), then the round's rocprofv3 profile of
# the headline command (kernel trace/stats, PMC passes one counter set per run)
set -u
O=gpurun_out/r04k
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_tier1.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1" \
  "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1" \
  "timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err" \
  "BATCHES='1024 4096' timeout -k 10 300 bash scripts/batch_sweep.sh r04k/v6ps0 > /dev/null 2>&1" \
  "TFHE_AMD_V6_PAIRSYNC=1 BATCHES='1024 4096' timeout -k 10 300 bash scripts/batch_sweep.sh r04k/v6ps1 > /dev/null 2>&1" \
  "timeout -k 10 1000 bash scripts/profile_round.sh r04k > $O/profile.txt 2>&1"
