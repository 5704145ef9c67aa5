#!/usr/bin/env bash
# GPU box: matrix-core counters of the int8 MFMA key switch (ks-v5) in the default bench (own run)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_ks5
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 5 --warmup 1 --batch ${1:-1024} --no-cpu-baseline --no-clock --no-ceiling --extra-batches none --strong-batch 0"
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS --output-format csv -d "$OUT/a" -o run -- python3 $BENCH > "$OUT/a.log" 2>&1 || exit 3
echo done
