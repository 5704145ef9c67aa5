"""Generate the golden fixtures in tests/golden/ from the reference's OWN compiled leaf
sources (oracle/_ref/libtfheref.so, built by oracle/build_ref.sh from
/root/reference/gpuParallel/{numeric-functions,multiplication,lwe-functions,...,tgsw,tlwe,
lwekeyswitch}.cu).

Run in the build container (the reference is not on the GPU box):
    oracle/build_ref.sh && python tests/golden/make_golden.py
Writes tests/golden/ref_leaf_vectors.npz (data only: inputs + reference outputs).
"""
import ctypes
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(REPO, "oracle", "_ref", "libtfheref.so")

N = 1024
I32P = ctypes.POINTER(ctypes.c_int32)


def p(a):
    return a.ctypes.data_as(I32P)


def main():
    ref = ctypes.CDLL(LIB)
    ref.ref_modswitch_to.restype = ctypes.c_int32
    rng = np.random.default_rng(20201015)
    out = {}

    # (1) exact negacyclic products: multiplication.cu naive and Karatsuba
    digs, polys, naive, kara, acc_in, acc_out = [], [], [], [], [], []
    cases = 6
    for c in range(cases):
        d = rng.integers(-512, 512, N, dtype=np.int64).astype(np.int32)
        q = rng.integers(-2**31, 2**31, N, dtype=np.int64).astype(np.int32)
        if c == 4:      # extremes
            d[:] = -512
            q[:] = np.int32(-2**31)
        if c == 5:
            d[:] = 511
            q[:] = np.int32(2**31 - 1)
        r1 = np.zeros(N, np.int32)
        r2 = np.zeros(N, np.int32)
        ref.ref_mult_naive(p(r1), p(d), p(q), N)
        ref.ref_mult_karatsuba(p(r2), p(d), p(q), N)
        a0 = rng.integers(-2**31, 2**31, N, dtype=np.int64).astype(np.int32)
        a1 = a0.copy()
        ref.ref_addmul_karatsuba(p(a1), p(d), p(q), N)
        digs.append(d); polys.append(q); naive.append(r1); kara.append(r2)
        acc_in.append(a0); acc_out.append(a1)
    out["mul_dig"] = np.stack(digs)
    out["mul_poly"] = np.stack(polys)
    out["mul_naive"] = np.stack(naive)
    out["mul_karatsuba"] = np.stack(kara)
    out["addmul_in"] = np.stack(acc_in)
    out["addmul_out"] = np.stack(acc_out)

    # (2) modSwitchFromTorus32 including the Msize edge (returns 2048 near 2^32)
    edge = [0, 1, -1, 2**31 - 1, -2**31, 2**20, -2**20, -2**20 - 1, -2**20 + 1,
            2**21, 2**21 - 1, 2**21 + 1, 3 * 2**20, 3 * 2**20 - 1, 2**29, -2**29]
    xs = np.concatenate([np.array(edge, np.int64),
                         rng.integers(-2**31, 2**31, 4000, dtype=np.int64)]).astype(np.int32)
    out["ms_x"] = xs
    for M in (2048, 8, 4, 1024):
        o = np.zeros_like(xs)
        ref.ref_modswitch_from(p(o), p(xs), len(xs), M)
        out[f"ms_from_{M}"] = o
    pairs = [(1, 8), (-1, 8), (1, 4), (-1, 4), (0, 8), (3, 8), (1, 2048), (-5, 2048)]
    out["ms_to_pairs"] = np.array(pairs, np.int32)
    out["ms_to"] = np.array([ref.ref_modswitch_to(m, M) for m, M in pairs], np.int32)

    # (3) the reference RNG: seed {314,1592,657} (cpuParallel/main.cpp:21-22), LWE key
    # n=500 (lweKeyGen) and 16 encryptions (lweSymEncrypt) of +-1/8 with ks_stdev
    seed = np.array([314, 1592, 657], np.uint32)
    n = 500
    alpha = math.sqrt(2.0 / math.pi) * 2.0 ** -15
    mu = np.array([ref.ref_modswitch_to(1 if (i % 3) else -1, 8) for i in range(16)], np.int32)
    key = np.zeros(n, np.int32)
    a = np.zeros((16, n), np.int32)
    b = np.zeros(16, np.int32)
    ref.ref_lwe_keygen_encrypt(seed.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 3, n,
                               ctypes.c_double(alpha), p(mu), 16, p(key), p(a), p(b))
    out["enc_seed"] = seed
    out["enc_mu"] = mu
    out["enc_key"] = key
    out["enc_a"] = a
    out["enc_b"] = b

    # (4) LWE ops
    ops_in_r = rng.integers(-2**31, 2**31, (6, n), dtype=np.int64).astype(np.int32)
    ops_in_s = rng.integers(-2**31, 2**31, (6, n), dtype=np.int64).astype(np.int32)
    rb = rng.integers(-2**31, 2**31, 6, dtype=np.int64).astype(np.int32)
    sb = rng.integers(-2**31, 2**31, 6, dtype=np.int64).astype(np.int32)
    pp = np.array([ref.ref_modswitch_to(1, 8), 0, 0, 2, 2, 0], np.int32)
    oa = ops_in_r.copy()
    ob = rb.copy()
    for op in range(6):
        r_b = ctypes.c_int32(int(ob[op]))
        row = np.ascontiguousarray(oa[op])
        ref.ref_lwe_op(op, n, p(row), ctypes.byref(r_b), p(np.ascontiguousarray(ops_in_s[op])),
                       ctypes.c_int32(int(sb[op])), int(pp[op]))
        oa[op] = row
        ob[op] = r_b.value
    out["lweop_r_a"] = ops_in_r
    out["lweop_r_b"] = rb
    out["lweop_s_a"] = ops_in_s
    out["lweop_s_b"] = sb
    out["lweop_p"] = pp
    out["lweop_out_a"] = oa
    out["lweop_out_b"] = ob

    # (5) gadget decomposition constants (tgsw.cu:7-29 over tlwe.cu's TLweParams) and the
    # key-switching key index map (lwekeyswitch.cu:3-18) at the default parameters
    h = np.zeros(2, np.int32)
    off = ctypes.c_uint32(0)
    ints = np.zeros(4, np.int32)
    ref.ref_tgsw_params(2, 10, N, 1, p(h), ctypes.byref(off), p(ints))
    out["tgsw_h"] = h
    out["tgsw_offset"] = np.array([off.value], np.uint32)
    out["tgsw_kpl_bg_halfbg_maskmod"] = ints
    idx = np.zeros(N * 8 * 4, np.int32)
    ref.ref_ksk_index(N, 8, 2, p(idx))
    out["ksk_index"] = idx

    # (6) struct layouts of the reference's own headers (oracle/ref_layout.cpp)
    import json
    import subprocess
    lay = subprocess.check_output([os.path.join(REPO, "oracle", "_ref", "ref_layout")]).decode()
    with open(os.path.join(HERE, "abi_layout.json"), "w") as f:
        json.dump(json.loads(lay), f, indent=1, sort_keys=True)

    path = os.path.join(HERE, "ref_leaf_vectors.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
