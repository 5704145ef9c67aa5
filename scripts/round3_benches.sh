#!/usr/bin/env bash
# GPU box: the config 3-5 benches on the current engine (profiles/r03_*)
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u bench_circuits.py > gpurun_out/r03_circuits.jsonl 2> gpurun_out/r03_circuits.err || exit $?
timeout -k 10 200 python -u bench_matvec.py > gpurun_out/r03_matvec.jsonl 2> gpurun_out/r03_matvec.err || exit $?
timeout -k 10 200 python -u bench_matvec.py --multi 0 >> gpurun_out/r03_matvec.jsonl 2>> gpurun_out/r03_matvec.err || exit $?
timeout -k 10 200 python -u bench_matvec.py --multi 0,0 >> gpurun_out/r03_matvec.jsonl 2>> gpurun_out/r03_matvec.err || exit $?
timeout -k 10 200 python -u bench_matvec.py --rank-of 0 --world-of 8 --reps 2 >> gpurun_out/r03_matvec.jsonl 2>> gpurun_out/r03_matvec.err || exit $?
timeout -k 10 300 python -u bench_matmat.py > gpurun_out/r03_matmat.jsonl 2> gpurun_out/r03_matmat.err || exit $?
exit 0
