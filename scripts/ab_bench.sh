#!/usr/bin/env bash
# A/B of library variants in one GPU session: scripts/ab_bench.sh name1 name2 ... ("base" = lib/)
# (AB_BATCH, AB_REPS, AB_STEPS, AB_WARMUP).  One summary line per run in gpurun_out/ab_summary.txt.
set -u
mkdir -p gpurun_out
for rep in $(seq 1 ${AB_REPS:-1}); do
for n in "$@"; do
  # "base" = lib/ (default kernel), "brN" = lib/ with TFHE_AMD_BR=N, "noguard" = lib/ with
  # TFHE_AMD_GUARD=0, "v10" / "v10all" = lib/ with TFHE_AMD_V10=1 / 2, "pair" = lib/
# with TFHE_AMD_V6_PAIR=1, "<variant>+v10" = variants/<variant>/ with TFHE_AMD_V10=1, "<variant>-ng" = variants/<variant>/ with TFHE_AMD_GUARD=0, else variants/<name>/
  br=0; guard=1; v10=0; pair=
  case "$n" in
    base) lib=cpu-gpu-tfhe_amd/lib/libtfhe_amd.so ;;
    v10) lib=cpu-gpu-tfhe_amd/lib/libtfhe_amd.so; v10=1 ;;
    v10all) lib=cpu-gpu-tfhe_amd/lib/libtfhe_amd.so; v10=2 ;;
    pair) lib=cpu-gpu-tfhe_amd/lib/libtfhe_amd.so; pair=1 ;;
    *+v10) lib=cpu-gpu-tfhe_amd/variants/${n%+v10}/libtfhe_amd.so; v10=1 ;;
    noguard) lib=cpu-gpu-tfhe_amd/lib/libtfhe_amd.so; guard=0 ;;
    *-ng) lib=cpu-gpu-tfhe_amd/variants/${n%-ng}/libtfhe_amd.so; guard=0 ;;
    br*) lib=cpu-gpu-tfhe_amd/lib/libtfhe_amd.so; br=${n#br} ;;
    *) lib=cpu-gpu-tfhe_amd/variants/$n/libtfhe_amd.so ;;
  esac
  log=gpurun_out/ab_${n}_${AB_BATCH:-1024}_$rep.log
  xenv=(); [ -n "$pair" ] && xenv=(TFHE_AMD_V6_PAIR=$pair)
  env "${xenv[@]}" TFHE_AMD_V10=$v10 TFHE_AMD_GUARD=$guard TFHE_AMD_BR=$br TFHE_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps ${AB_STEPS:-5} --warmup ${AB_WARMUP:-1} --batch ${AB_BATCH:-1024} --no-cpu-baseline --no-clock --no-ceiling --extra-batches '' --strong-batch 0 > $log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -5 $log; exit $rc; }
  python3 -c "
import json,sys
d=[json.loads(l) for l in open('$log') if l.startswith('{')][-1]
print('%-10s B=%-5s rep %s  %9.0f /s  br %.3f ms  ks %.3f ms  ok=%s' % ('$n', '${AB_BATCH:-1024}', $rep, d['value'], d['roofline']['kernel_ms'], d['roofline']['keyswitch_ms'], d['truth_table_ok']))" | tee -a gpurun_out/ab_summary.txt
done
done
exit 0
