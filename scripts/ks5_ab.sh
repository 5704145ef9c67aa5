set -u
for B in 1024 4096 128 256 512; do
for m in 0 1; do
  TFHE_AMD_KS5=$m timeout -k 10 200 python bench.py --steps 10 --warmup 2 --batch $B --no-cpu-baseline --no-clock --no-ceiling --extra-batches '' --strong-batch 0 > gpurun_out/ksab_${B}_$m.json 2>&1 || exit 1
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/ksab_${B}_$m.json') if l.startswith('{')][-1]
print('B=$B ks5=$m  %.0f /s  br %.3f ks %.3f ms ok=%s' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['keyswitch_ms'], d['truth_table_ok']))"
done; done
