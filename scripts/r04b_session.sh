#!/usr/bin/env bash
# (historical record of a round-4 session: it ran variants since retired — v9 / the one-wave key-prefetch build — and is kept with the profiles it produced, not for re-running)
# GPU box, round 4: new/changed tests, the v9 A/B sweep, the Tier-1 queue rate, the host-path
# rate and the host copy micro-benchmark (each step under its own time limit; stops on a fault)
set -u
O=gpurun_out/r04b
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 500 python -u -m pytest tests/test_v9.py tests/test_l1_exports.py tests/test_multi_gpu.py tests/test_circuits.py tests/test_tier1.py tests/test_gpu_parity.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/tests.txt 2>&1" \
  "BATCHES='1 64 256 512' timeout -k 10 400 bash scripts/batch_sweep.sh r04b/v6 > /dev/null 2>&1" \
  "TFHE_AMD_V9=1 BATCHES='1 64 256 512' timeout -k 10 400 bash scripts/batch_sweep.sh r04b/v9 > /dev/null 2>&1" \
  "timeout -k 10 200 tests/callers/_bin/tier1_rate 16 1 8 64 > $O/tier1_rate.json 2>&1" \
  "timeout -k 10 200 python scripts/host_path_rate.py 1 1024 2048 4096 > $O/host_path.jsonl 2>&1" \
  "timeout -k 10 120 scripts/host_copy_ubench 1024 > $O/copy_1024.jsonl 2>&1" \
  "timeout -k 10 120 scripts/host_copy_ubench 4096 > $O/copy_4096.jsonl 2>&1"
