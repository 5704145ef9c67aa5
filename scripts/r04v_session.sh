#!/usr/bin/env bash
# GPU box, round 4 session v: the N > 1 bench path rehearsed with two ranks sharing the one GPU
# (gloo for the timing reductions), as the driver's torchrun launch
set -u
O=gpurun_out/r04v
mkdir -p $O
bash scripts/gpu_session.sh \
  "TFHE_AMD_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_2ranks.json 2> $O/bench_2ranks.err"
