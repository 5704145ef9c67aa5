#!/usr/bin/env bash
# GPU box: parity suite, default bench line, batch table, circuits, matvec, rocprof profiles
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
bash scripts/bench_table.sh || exit 3
timeout -k 10 400 python bench_circuits.py > gpurun_out/circ.jsonl 2> gpurun_out/circ.err || exit 3
timeout -k 10 300 python bench_matvec.py > gpurun_out/mv64.jsonl 2> gpurun_out/mv.err || exit 3
timeout -k 10 200 python bench_matvec.py --rank-of 0 --world-of 8 --reps 2 > gpurun_out/mv8.jsonl 2>> gpurun_out/mv.err || exit 3
bash scripts/profile_round.sh ${1:-final} 1024
