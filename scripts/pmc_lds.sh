#!/usr/bin/env bash
# LDS / VALU occupancy counters of the default bench (GPU box): scripts/pmc_lds.sh <tag>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 2 --warmup 1 --batch ${BATCH:-1024} --no-cpu-baseline"
i=0
for set in "SQ_BUSY_CYCLES SQ_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL" \
           "SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL" \
           "SQ_INSTS_LDS_STORE_BANDWIDTH SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o run -- python3 $BENCH > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
