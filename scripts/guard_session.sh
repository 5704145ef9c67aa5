#!/usr/bin/env bash
# GPU box: parity suite, then the guard's cost: base (guarded) vs TFHE_AMD_GUARD=0 (no flags /
# exact-kernel launch) vs the build without the in-loop rounding-distance check.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error|distance" gpurun_out/pytest_gpu.log | tail -5; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/ab_summary.txt
AB_REPS=3 AB_STEPS=10 bash scripts/ab_bench.sh base noguard noguard_build-ng || exit 3
AB_BATCH=4096 AB_STEPS=5 bash scripts/ab_bench.sh base noguard_build-ng || exit 3
AB_BATCH=1 AB_STEPS=20 bash scripts/ab_bench.sh base noguard_build-ng || exit 3
