#!/usr/bin/env bash
# GPU box: the config 3-5 benches on the current engine (profiles/r03_*)
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u bench_circuits.py > gpurun_out/${TAG:-r03}_circuits.jsonl 2> gpurun_out/${TAG:-r03}_circuits.err || exit $?
timeout -k 10 200 python -u bench_matvec.py > gpurun_out/${TAG:-r03}_matvec.jsonl 2> gpurun_out/${TAG:-r03}_matvec.err || exit $?
timeout -k 10 200 python -u bench_matvec.py --multi 0 >> gpurun_out/${TAG:-r03}_matvec.jsonl 2>> gpurun_out/${TAG:-r03}_matvec.err || exit $?
timeout -k 10 200 python -u bench_matvec.py --multi 0,0 >> gpurun_out/${TAG:-r03}_matvec.jsonl 2>> gpurun_out/${TAG:-r03}_matvec.err || exit $?
timeout -k 10 200 python -u bench_matvec.py --rank-of 0 --world-of 8 --reps 2 >> gpurun_out/${TAG:-r03}_matvec.jsonl 2>> gpurun_out/${TAG:-r03}_matvec.err || exit $?
timeout -k 10 300 python -u bench_matmat.py > gpurun_out/${TAG:-r03}_matmat.jsonl 2> gpurun_out/${TAG:-r03}_matmat.err || exit $?
exit 0
