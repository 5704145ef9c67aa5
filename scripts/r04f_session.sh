#!/usr/bin/env bash
# (historical record of a round-4 session: it ran variants since retired — v9 / the one-wave key-prefetch build — and is kept with the profiles it produced, not for re-running)
# GPU box, round 4 session f: (1) the host copy pool + pinned readback (host path, LweSample batch,
# Tier-1 queue with its per-phase times), (2) the paired kernel's one-wave build with a whole step
# of key prefetch (TFHE_AMD_V6P_PF=1): parity, then an A/B at the batches it serves
set -u
O=gpurun_out/r04f
R=$(pwd)
mkdir -p $O
bash scripts/gpu_session.sh \
  "timeout -k 10 400 python -u -m pytest tests/test_tier1.py tests/test_gpu_parity.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/tests.txt 2>&1" \
  "timeout -k 10 200 python scripts/host_path_rate.py 1 64 1024 2048 4096 > $O/host_path.jsonl 2>&1" \
  "timeout -k 10 200 tests/callers/_bin/tier1_rate 16 1 8 64 > $O/tier1_rate.json 2>&1" \
  "TFHE_AMD_V6P_PF=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k 'paired or gate_batch or mux or woks' > $O/tests_pf.txt 2>&1" \
  "BATCHES='512 384' timeout -k 10 300 bash scripts/batch_sweep.sh r04f/pf0 > /dev/null 2>&1" \
  "TFHE_AMD_V6P_PF=1 BATCHES='512 384' timeout -k 10 300 bash scripts/batch_sweep.sh r04f/pf1 > /dev/null 2>&1" \
  "BATCHES='512' timeout -k 10 300 bash scripts/batch_sweep.sh r04f/pf0b > /dev/null 2>&1" \
  "TFHE_AMD_V6P_PF=1 BATCHES='512' timeout -k 10 300 bash scripts/batch_sweep.sh r04f/pf1b > /dev/null 2>&1" \
  "cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/tr -o run -- python3 $R/scripts/host_path_rate.py 1024 4096 > $R/$O/host_path_traced.jsonl 2>&1"
