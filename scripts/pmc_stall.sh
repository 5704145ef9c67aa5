#!/usr/bin/env bash
# GPU box: where the blind-rotation waves wait (two SQ passes, kernel trace only, own runs each)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-stall}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 5 --warmup 1 --batch ${2:-1024} --no-cpu-baseline --no-clock --no-ceiling --extra-batches none --strong-batch 0"
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --output-format csv -d "$OUT/a" -o run -- python3 $BENCH > "$OUT/a.log" 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_MISC --output-format csv -d "$OUT/b" -o run -- python3 $BENCH > "$OUT/b.log" 2>&1 || exit 4
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES --output-format csv -d "$OUT/c" -o run -- python3 $BENCH > "$OUT/c.log" 2>&1 || exit 5
echo done
