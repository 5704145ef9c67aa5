#!/usr/bin/env bash
# Runs on the GPU box (gpurun): rocprofv3 kernel trace/stats of the default bench, then the
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters) each in its own run, kernel-trace only.
#   bash scripts/profile_round.sh <tag> [batch]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
BATCH=${2:-1024}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# the bench's own warm-up (10) and step count (20), so that the profiler's average of the blind
# rotation is over settled launches like the line's kernel_ms (scripts/trace_mean.py compares them)
BENCH="$R/bench.py --steps 20 --warmup 10 --batch $BATCH --no-cpu-baseline --no-clock --no-ceiling --extra-batches none --strong-batch 0 --parity-samples 0"
run() {   # name, extra rocprofv3 args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 $BENCH > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run trace --kernel-trace --stats
python3 "$R/scripts/trace_mean.py" "$(find "$OUT/trace" -name '*kernel_trace.csv' | head -n 1)" \
    "$(find "$OUT/trace" -name '*kernel_stats.csv' | head -n 1)" "$OUT/trace.log" 20 > "$OUT/trace_mean.json" 2>&1 || true
run fetch --kernel-trace --pmc FETCH_SIZE
run write --kernel-trace --pmc WRITE_SIZE
run sq --kernel-trace --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY
run sq2 --kernel-trace --pmc SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_WAVES
run l2 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum
run lds --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT
exit 0
