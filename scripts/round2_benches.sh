#!/usr/bin/env bash
# GPU box: circuit / matrix-vector / matrix-product benches of this round -> gpurun_out/r02_*.jsonl
set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench_circuits.py --reps 3 > gpurun_out/r02_circuits.jsonl 2> gpurun_out/r02_circuits.err || exit 3
for s in 4 8 16; do
  timeout -k 10 300 python bench_matmat.py --size $s >> gpurun_out/r02_matmat.jsonl 2>> gpurun_out/r02_matmat.err || exit 4
done
timeout -k 10 300 python bench_matvec.py >> gpurun_out/r02_matvec.jsonl 2>> gpurun_out/r02_matvec.err || exit 5
timeout -k 10 300 python bench_matvec.py --rank-of 0 --world-of 8 >> gpurun_out/r02_matvec.jsonl 2>> gpurun_out/r02_matvec.err || exit 5
cat gpurun_out/r02_circuits.jsonl gpurun_out/r02_matmat.jsonl gpurun_out/r02_matvec.jsonl | cut -c1-260
