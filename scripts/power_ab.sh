#!/usr/bin/env bash
# Time AND power of library variants (GPU box, diagnostics): for each variant a long bench run
# at batch PB (default 1024) while amd-smi samples socket power and the GFX clock; one summary
# line per variant in gpurun_out/power_ab.txt (blind-rotation ms, mean W, mean MHz, J per launch).
#   scripts/power_ab.sh name1 name2 ...   ("base" = lib/, "noguard" = lib/ with the guard off,
#                                          "<v>-ng" = variants/<v>/ with the guard off (timing
#                                          diagnostics give wrong results), else variants/<name>/)
set -u
mkdir -p gpurun_out
B=${PB:-1024}
for n in "$@"; do
  guard=1
  case "$n" in
    base) lib=cpu-gpu-tfhe_amd/lib/libtfhe_amd.so ;;
    noguard) lib=cpu-gpu-tfhe_amd/lib/libtfhe_amd.so; guard=0 ;;
    *-ng) lib=cpu-gpu-tfhe_amd/variants/${n%-ng}/libtfhe_amd.so; guard=0 ;;
    *) lib=cpu-gpu-tfhe_amd/variants/$n/libtfhe_amd.so ;;
  esac
  log=gpurun_out/pw_${n}_$B.json
  smp=gpurun_out/pw_${n}_$B.smi
  : > $smp
  TFHE_AMD_GUARD=$guard TFHE_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps ${PSTEPS:-4000} --warmup 2 \
      --batch $B --no-cpu-baseline --no-clock --no-ceiling --extra-batches '' --strong-batch 0 > $log 2>&1 &
  pid=$!
  sleep ${PDELAY:-4}
  for k in $(seq 1 8); do
    kill -0 $pid 2>/dev/null || break
    amd-smi metric -g 0 --clock --power 2>&1 | grep -E "SOCKET_POWER|^ *CLK:" | head -3 >> $smp
    sleep 0.7
  done
  wait $pid
  rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -5 $log; exit $rc; }
  python3 - "$n" "$log" "$smp" <<'EOF' | tee -a gpurun_out/power_ab.txt
import json, re, sys
n, log, smp = sys.argv[1:]
d = [json.loads(l) for l in open(log) if l.startswith('{')][-1]
txt = open(smp).read()
w = [float(x) for x in re.findall(r'SOCKET_POWER:\s*([0-9.]+)', txt)]
c = [float(x) for x in re.findall(r'CLK:\s*([0-9.]+)', txt)]
w = [x for x in w if x > 400] or [0.0]
c = [x for x in c if x > 600] or [0.0]
W = sum(w) / len(w)
ms = d['roofline']['kernel_ms']
step = d['ms_per_step']
print('%-8s B=%s br %.3f ms  step %.3f ms  %5.0f W  %5.0f MHz  %.2f J/step  (%d W samples)' %
      (n, d['config']['batch_per_gpu'], ms, step, W, sum(c) / len(c), W * step / 1000, len(w)))
EOF
done
exit 0
