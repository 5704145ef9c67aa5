#!/usr/bin/env bash
# A/B of library variants in one GPU session: scripts/ab_bench.sh name1 name2 ... ("base" = lib/)
set -u
for n in "$@"; do
  if [ "$n" = base ]; then lib=cpu-gpu-tfhe_amd/lib/libtfhe_amd.so; else lib=cpu-gpu-tfhe_amd/variants/$n/libtfhe_amd.so; fi
  TFHE_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps 3 --warmup 1 --batch ${AB_BATCH:-1024} --no-cpu-baseline > gpurun_out/ab_${n}_${AB_BATCH:-1024}.log 2>&1
  rc=$?; echo "$n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
