"""bench_circuits.py — BASELINE.json configs 3 and 4 on the batched circuit engine (§8(f) row 1).

  config 3: 32-bit ripple-carry encrypted addition (Cipher.cpp operator+ path)
  config 4: 16-bit x 16-bit encrypted multiplication, batch 256 (multiplyLweSamples path)
  plus Cipher's other operators as circuits: signed >, ==, minimum, signed division (16-bit)

Each circuit is built once (csrc/circuit.cpp), inputs are encrypted under the seeded keys and
resident in HBM, and the timed region is the whole circuit evaluation (every level's blind
rotation + key switch launches) between torch.cuda.synchronize() calls; results are decrypted
afterwards and checked against integer arithmetic.  Prints one JSON line per measurement.

    python bench_circuits.py [--reps R] [--quick]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cpu-gpu-tfhe_amd"))


def run_case(T, torch, ctx, K, name, build, nbits, B, reps, rng, ref):
    C = T.Circuit()
    a, b = C.inputs(nbits), C.inputs(nbits)
    outs = build(C, a, b)
    info = C.info()
    x = rng.integers(0, 2**nbits, B)
    y = rng.integers(0, 2**nbits, B)
    n_w = info["wires"]
    wa = torch.zeros((n_w, B, 500), dtype=torch.int32, device="cuda")
    wb = torch.zeros((n_w, B), dtype=torch.int32, device="cuda")
    for wires, v in ((a, x), (b, y)):
        for w, plane in zip(wires, T.bits_of(v, nbits)):
            ea, eb = K.encrypt(plane, rng)
            wa[w] = torch.from_numpy(ea).cuda()
            wb[w] = torch.from_numpy(eb).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    C.run_dev(ctx, B, wa, wb, stream)                     # warm-up (compiles + uploads tables)
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        C.run_dev(ctx, B, wa, wb, stream)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    ha, hb = wa.cpu().numpy(), wb.cpu().numpy()
    got = T.int_of([K.decrypt(ha[w], hb[w]) for w in outs])
    ok = bool(np.array_equal(got, ref(x, y)))
    t = float(np.median(times))
    return {"case": name, "nbits": nbits, "batch": B, "seconds": t, "per_instance_s": t / B,
            "bootstraps_per_instance": info["bootstraps"], "depth": info["depth"],
            "bootstraps_per_s": info["bootstraps"] * B / t, "correct": ok, "reps": reps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--quick", action="store_true", help="smaller batches (smoke)")
    args = ap.parse_args()
    import torch
    import tfhe_amd as T
    torch.cuda.set_device(0)
    K = T.SecretKeyset()
    ctx = T.Context(K.bk, K.ksk, device=0)
    rng = np.random.default_rng(7)
    add = (lambda x, y: x + y)

    def sgn(v):
        v = np.asarray(v, dtype=np.int64)
        return np.where(v >= 2**15, v - 2**16, v)

    def sdiv(x, y):   # truncation toward zero, mod 2^16 (y = 0 gives what the circuit gives: skipped)
        xs, ys = sgn(x), sgn(y)
        q = [(-1 if (p < 0) != (d < 0) else 1) * (abs(int(p)) // abs(int(d))) if d else -1 for p, d in zip(xs, ys)]
        return np.array(q, dtype=np.int64) % 2**16

    def ripple(C, a, b):
        s, co = C.add(a, b)
        return s + [co]

    def prefix(C, a, b):
        s, co = C.add_prefix(a, b)
        return s + [co]

    cases = [
        ("config3: 32-bit ripple-carry add", ripple, 32, 1, add),
        ("32-bit ripple-carry add, batch 1024", ripple, 32, 1024 if not args.quick else 64, add),
        ("32-bit parallel-prefix add", prefix, 32, 1, add),
        ("config4: 16x16 multiply, batch 256", lambda C, a, b: C.mul(a, b), 16, 256 if not args.quick else 16,
         lambda x, y: x * y),
        ("16x16 multiply, batch 1", lambda C, a, b: C.mul(a, b), 16, 1, lambda x, y: x * y),
        ("16-bit signed a > b (operator>)", lambda C, a, b: [C.compare(a, b, "GT", True)], 16, 1,
         lambda x, y: (sgn(x) > sgn(y)).astype(np.int64)),
        ("16-bit a == b (operator==)", lambda C, a, b: [C.compare(a, b, "EQ")], 16, 1,
         lambda x, y: (x == y).astype(np.int64)),
        ("16-bit minimum", lambda C, a, b: C.minmax(a, b), 16, 1, np.minimum),
        ("16-bit signed division (operator/)", lambda C, a, b: C.div(a, b), 16, 1, sdiv),
        ("16-bit signed division, batch 256", lambda C, a, b: C.div(a, b), 16, 256 if not args.quick else 16,
         sdiv),
    ]
    for name, build, nbits, B, ref in cases:
        r = run_case(T, torch, ctx, K, name, build, nbits, B, args.reps, rng, ref)
        r["engine"] = T.version()
        print(json.dumps(r), flush=True)
    ctx.close()
    K.close()


if __name__ == "__main__":
    main()
