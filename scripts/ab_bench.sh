#!/usr/bin/env bash
# A/B of library builds in one GPU session: scripts/ab_bench.sh name1 name2 ...
#   "base" = cpu-gpu-tfhe_amd/lib/ (the product build), any other name = cpu-gpu-tfhe_amd/variants/<name>/
#   (built with: make -C cpu-gpu-tfhe_amd BUILD=build_<name> LIB=variants/<name>/libtfhe_amd.so EXTRA=...)
# (AB_BATCH, AB_REPS, AB_STEPS, AB_WARMUP).  One summary line per run in gpurun_out/ab_summary.txt;
# the names alternate within each repetition, so every pair ran on the same box, back to back.
set -u
mkdir -p gpurun_out
for rep in $(seq 1 ${AB_REPS:-1}); do
for n in "$@"; do
  case "$n" in
    base) lib=cpu-gpu-tfhe_amd/lib/libtfhe_amd.so ;;
    *) lib=cpu-gpu-tfhe_amd/variants/$n/libtfhe_amd.so ;;
  esac
  log=gpurun_out/ab_${n}_${AB_BATCH:-1024}_$rep.log
  TFHE_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps ${AB_STEPS:-5} --warmup ${AB_WARMUP:-1} \
      --batch ${AB_BATCH:-1024} --no-cpu-baseline --no-clock --no-ceiling --no-circuits --extra-batches none \
      --strong-batch none --host-batches none > $log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -5 $log; exit $rc; }
  python3 -c "
import json,sys
d=[json.loads(l) for l in open('$log') if l.startswith('{')][-1]
print('%-10s B=%-5s rep %s  %9.0f /s  %.3f ms/step  br %.3f ms  ks %.3f ms  ok=%s parity=%s' % ('$n', '${AB_BATCH:-1024}', $rep, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['keyswitch_ms'], d['truth_table_ok'], d['parity']['mismatches']))" | tee -a gpurun_out/ab_summary.txt
done
done
exit 0
