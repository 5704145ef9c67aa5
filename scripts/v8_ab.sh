#!/usr/bin/env bash
# GPU box: v8 (4 waves per ciphertext; EXPERIMENTAL=1 builds only since it lost) parity vs the oracle,
# then bench lines with and without it
#   bash scripts/v8_ab.sh <tag>
set -u
TAG=${1:-v8}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 240 env TFHE_AMD_V8=1 python -u - > "$OUT/parity.txt" 2>&1 <<'PY'
import sys, numpy as np
sys.path[:0] = ["cpu-gpu-tfhe_amd", "tests"]
import tfhe_amd as T, oracle_ctypes as O
K = T.SecretKeyset(); c = T.Context(K.bk, K.ksk, device=0); o = O.OracleKey(K.bk, K.ksk, use_ntt=True)
rng = np.random.default_rng(3)
for gate, B in (("NAND", 300), ("XOR", 1), ("AND", 512), ("MUX", 40)):
    bits = [rng.integers(0, 2, B) for _ in range(3 if gate == "MUX" else 2)]
    host = [v for b in bits for v in K.encrypt(b, rng)]
    r = c.gate_host(gate, *host)
    kern = c.last_kernels()
    idx = np.unique(np.concatenate([[0, B - 1], rng.choice(B, min(B, 48), replace=False)]))
    w = o.gate_batch(gate, *(v[idx] for v in host))
    bad = int(np.sum(np.any(r[0][idx] != w[0], axis=1) | (r[1][idx] != w[1])))
    tt = {"NAND": lambda x, y: 1 - (x & y), "XOR": lambda x, y: x ^ y, "AND": lambda x, y: x & y}
    want = np.where(bits[0] == 1, bits[1], bits[2]) if gate == "MUX" else tt[gate](bits[0], bits[1])
    dec = np.array_equal(K.decrypt(*r), want)
    print(gate, B, "sampled", len(idx), "mismatches", bad, "decrypt_ok", dec, kern, flush=True)
    assert bad == 0 and dec
print("guard", c.guard_stats())
print("v8 parity ok")
PY
rc=$?; echo "parity rc=$rc"; [ $rc -ne 0 ] && exit $rc
for v in 0 1; do
  timeout -k 10 240 env TFHE_AMD_V8=$v python -u bench.py --batch 512 --steps 20 --warmup 5 --extra-batches 256,1,300,400 \
      --strong-batch 0 --no-cpu-baseline --no-clock --no-ceiling --parity-samples 32 > "$OUT/bench_v8_$v.json" 2> "$OUT/bench_v8_$v.err"
  rc=$?; echo "bench v8=$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
