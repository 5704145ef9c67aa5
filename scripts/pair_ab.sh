# A/B: one vs two ciphertexts per v6 workgroup (TFHE_AMD_V6_PAIR=0/1; unset = the default policy)
set -u
for B in ${BATCHES:-256 512 768 1024 2048 4096}; do
for m in ${MODES:-0 1}; do
  if [ "$m" = def ]; then unset TFHE_AMD_V6_PAIR; else export TFHE_AMD_V6_PAIR=$m; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 5 --batch $B --no-cpu-baseline --no-clock --no-ceiling --extra-batches '' --strong-batch 0 > gpurun_out/pairab_${B}_$m.json 2>&1 || exit 1
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/pairab_${B}_$m.json') if l.startswith('{')][-1]
print('B=$B pair=$m  %.0f /s  br %.3f ks %.3f ms ok=%s' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['keyswitch_ms'], d['truth_table_ok']))"
done; done
