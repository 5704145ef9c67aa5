#!/usr/bin/env bash
# Runs on the GPU box (gpurun): rocprofv3 of the bench line ITSELF — the driver's exact command,
# `python3 bench.py --gpus 1 --steps 20 --warmup 5` — under --kernel-trace --stats, then one PMC
# pass per counter set (each its own run, kernel-trace only), each pass again the same command.
# scripts/trace_mean.py pairs the run's own bench line (ms_per_step, kernel_ms, frac) with the
# rocprof durations of the headline's timed launches; scripts/pmc_summary.py turns the FETCH /
# WRITE passes of the same command into profiles/pmc_summary.json.
#   bash scripts/profile_round.sh <tag> [bench|headline] [extra bench args...]
#     bench    : the driver's command, every leg (default)
#     headline : only the B = 1024 headline (legs, CPU baseline, clock, ceiling off): quicker PMC
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
MODE=${2:-bench}
shift; [ $# -gt 0 ] && shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
if [ "$MODE" = headline ]; then
  BENCH="$R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-clock --no-ceiling --extra-batches none --strong-batch 0 --host-batches none $*"
else
  BENCH="$R/bench.py --gpus 1 --steps 20 --warmup 5 $*"
fi
# PMC passes: the same command with --no-clock — amd-smi is a python script started through
# /usr/bin/env, an exec the box refuses once the PMC profiler's preload has initialised the GPU
# (round-5 session r05a: the refused execs left the write pass hung); and --no-circuits: the PMC
# summaries read only the headline's launches, which come first
run() {   # name, extra rocprofv3 args...
  local name=$1; shift
  local extra=""
  case " $* " in *" --pmc "*) extra="--no-clock --no-circuits" ;; esac
  timeout -k 10 400 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 $BENCH $extra > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run trace --kernel-trace --stats
python3 "$R/scripts/trace_mean.py" "$(find "$OUT/trace" -name '*kernel_trace.csv' | head -n 1)" \
    "$(find "$OUT/trace" -name '*kernel_stats.csv' | head -n 1)" "$OUT/trace.log" 20 5 > "$OUT/trace_mean.json" 2>&1 || true
run fetch --kernel-trace --pmc FETCH_SIZE
run write --kernel-trace --pmc WRITE_SIZE
run sq --kernel-trace --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY
run sq2 --kernel-trace --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVES
run l2 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum
run lds --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT
exit 0
