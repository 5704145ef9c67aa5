"""Exactness guard of the fp64 FFT blind rotation (include/tfhe_amd.h
tfhe_amd_guard_stats).  The default kernel rounds each external-product coefficient to the
nearest integer, which is the exact product only while the FFT error stays below 1/2; every
launch measures the largest rounding distance per ciphertext and the exact 2-prime NTT kernel
recomputes the ones at or above 1/8 (or out of the shifter's range) before their key switch.

CPU: a constructed worst case — a bootstrapping key whose polynomials are all the constant
2^31 - 1 — drives the fp64 product's rounding distance to 1/2 in the numpy emulation of the
kernel's data flow (scripts/emu_v6.py) and in the fp64 CPU port, whose unguarded results are
then wrong on every coefficient, while real keys stay near 0.05.
GPU: with real keys nothing is recomputed and the distance stays below 1/8; with the threshold
forced to 0 every ciphertext (gates, MUX halves, circuit rows) is recomputed by the exact kernel
and the outputs are still the oracle's word for word; with the constructed key the guard fires
on its own and the outputs equal the oracle's exact ones; with random high-magnitude keys (not
constant) whose unguarded fp64 results are wrong on some ciphertexts and right on others, the
guarded results are all exact."""
import os
import sys

import numpy as np
import pytest

import oracle_ctypes as O
import tfhe_amd as T

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
import emu_v6 as E  # noqa: E402

MAXK = 2**31 - 1


def _emu_distance(d, bk):
    Tb = E.tables()
    acc = sum(E.fwd(d[p].astype(float), Tb) * (E.fwd(bk[p].astype(float), Tb) / 512) for p in range(4))
    c = E.inv_dit(acc)
    exact = np.array([int(x) for x in sum(E.negacyclic(d[p], bk[p]) for p in range(4))], dtype=object)
    wrong = int(np.sum(np.rint(c).astype(np.int64).astype(object) != exact))
    return float(np.max(np.abs(c - np.rint(c)))), wrong


def test_emulated_worst_case_key_trips_the_guard():
    r = np.random.default_rng(5)
    d = r.integers(-512, 512, (4, 1024))
    real, wrong_real = _emu_distance(d, r.integers(-2**31, 2**31, (4, 1024)))
    bad, _ = _emu_distance(np.full((4, 1024), -512), np.full((4, 1024), MAXK))
    assert real < 0.125 and wrong_real == 0
    assert bad >= 0.25, bad            # the guard's threshold: this step would be recomputed


def test_cpu_fft_port_worst_case_key(keyset, rng):
    """The same fp64 algorithm on the CPU with no guard: the constructed key makes it wrong."""
    B = 2
    x_a = rng.integers(-2**31, 2**31, (B, 500), dtype=np.int64).astype(np.int32)
    x_b = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
    bk = np.full_like(keyset.bk, MAXK)
    f = O.CpuFftKey(bk, keyset.ksk)
    got = f.woks_batch(1 << 29, x_a, x_b, nthreads=2)
    want = O.OracleKey(bk, keyset.ksk).woks_batch(1 << 29, x_a, x_b, nthreads=2)
    assert f.max_round_error() >= 0.25
    assert not np.array_equal(got[0], want[0])


# ---------------------------------------------------------------- GPU

@pytest.mark.gpu
def test_guard_quiet_on_real_keys(ctx, keyset, rng):
    ctx.guard_stats(reset=True)
    B = 256
    x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
    (a_a, a_b), (b_a, b_b) = keyset.encrypt(x, rng), keyset.encrypt(y, rng)
    r_a, r_b = ctx.gate_host("NAND", a_a, a_b, b_a, b_b)
    dist, redo = ctx.guard_stats(reset=True)
    print(f"largest rounding distance over {B} bootstraps: {dist:.4f}")
    assert redo == 0 and 0.0 < dist < 0.125
    assert np.array_equal(keyset.decrypt(r_a, r_b), 1 - (x & y))


@pytest.mark.gpu
def test_guard_forced_fallback_bit_exact(ctx, okey, keyset, rng):
    """Threshold 0: every blind rotation is recomputed by the exact kernel in guard mode —
    gates, both MUX halves, woKS and circuit rows — and the results are unchanged."""
    B = 12
    s, x, y = (rng.integers(0, 2, B) for _ in range(3))
    (sa, sb), (xa, xb), (ya, yb) = (keyset.encrypt(v, rng) for v in (s, x, y))
    ctx.guard_stats(reset=True)
    try:
        T.set_guard_threshold(0.0)
        g = ctx.gate_host("XOR", xa, xb, ya, yb)
        m = ctx.gate_host("MUX", sa, sb, xa, xb, ya, yb)
        u = ctx.woks_host(T.MU, xa, xb)
        _, redo = ctx.guard_stats(reset=True)
        C = T.Circuit()
        i0, i1, i2 = C.inputs(3)
        outs = [C.gate("MAJ", i0, i1, i2), C.gate("NAND", i0, i1)]
        got = C.run(ctx, B, {i0: s, i1: x, i2: y}, outs, keyset, rng)
        _, redo_c = ctx.guard_stats(reset=True)
    finally:
        T.set_guard_threshold(0.125)
    assert redo == B + 2 * B + B and redo_c == 2 * B
    assert all(np.array_equal(a, b) for a, b in zip(g, okey.gate_batch("XOR", xa, xb, ya, yb)))
    assert all(np.array_equal(a, b) for a, b in zip(m, okey.gate_batch("MUX", sa, sb, xa, xb, ya, yb)))
    assert all(np.array_equal(a, b) for a, b in zip(u, okey.woks_batch(T.MU, xa, xb)))
    assert np.array_equal(got[outs[0]], ((s + x + y) >= 2).astype(int))
    assert np.array_equal(got[outs[1]], 1 - (s & x))


@pytest.mark.gpu
def test_guard_forced_fallback_grid_stride(ctx, okey, keyset, rng):
    """More flagged ciphertexts than the guard launch has workgroups (256): each workgroup
    recomputes several in turn; every output still equals the oracle's."""
    B = 300
    x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
    (a_a, a_b), (b_a, b_b) = keyset.encrypt(x, rng), keyset.encrypt(y, rng)
    ctx.guard_stats(reset=True)
    try:
        T.set_guard_threshold(0.0)
        r = ctx.gate_host("OR", a_a, a_b, b_a, b_b)
        _, redo = ctx.guard_stats(reset=True)
    finally:
        T.set_guard_threshold(0.125)
    assert redo == B
    want = okey.gate_batch("OR", a_a, a_b, b_a, b_b)
    assert np.array_equal(r[0], want[0]) and np.array_equal(r[1], want[1])


@pytest.mark.gpu
def test_guard_catches_worst_case_key(keyset, rng):
    """The constructed key: the fp64 kernel's rounding distance reaches the threshold, the
    exact kernel recomputes those ciphertexts, and the woKS outputs equal the exact oracle's."""
    bk = np.full_like(keyset.bk, MAXK)
    B = 8
    x_a = rng.integers(-2**31, 2**31, (B, 500), dtype=np.int64).astype(np.int32)
    x_b = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
    c = T.Context(bk, keyset.ksk, device=0)
    try:
        u = c.woks_host(T.MU, x_a, x_b)
        dist, redo = c.guard_stats()
    finally:
        c.close()
    want = O.OracleKey(bk, keyset.ksk).woks_batch(T.MU, x_a, x_b)
    assert dist >= 0.125 and redo == B, (dist, redo)
    assert np.array_equal(u[0], want[0]) and np.array_equal(u[1], want[1])


def _torus_of_chk(c):
    """numpy restatement of csrc/fft_wave.h torus_of_chk (IEEE double; round 2's rounding, kept in
    the TFHE_AMD_V6_DISTGUARD A/B build and the experimental v8):
    returns (low word of y, rounding distance |c - q|, high word of y)."""
    c = np.asarray(c, dtype=np.float64)
    M2 = np.float64(1.5 * 2.0**52)
    y = c + M2
    q = y - M2
    bits = y.view(np.uint64)
    return (bits & 0xFFFFFFFF).astype(np.uint32), np.abs(c - q), (bits >> 32).astype(np.uint32)


def test_single_shifter_rounding_exact_or_flagged():
    """The kernel's mod-2^32 rounding (one 1.5 * 2^52 shifter) is exact for |c| < 2^51 and, over
    the whole product range |c| <= 2^52, either exact or flagged by the guard (distance >= 1/8,
    or the shifter's high word outside [hi(2^52), hi(2^53)), i.e. |c| >= 2^51)."""
    r = np.random.default_rng(9)
    mags = np.concatenate([r.uniform(-2.0**47, 2.0**47, 20000),
                           r.uniform(-2.0**52, 2.0**52, 20000),
                           r.uniform(2.0**50, 2.0**52, 5000) * r.choice([-1, 1], 5000)])
    fr = r.uniform(-0.49, 0.49, mags.shape)
    ints = np.floor(mags)
    c = ints + fr                                       # representable up to the ulp
    edges = np.array([2.0**51 - 1, 2.0**51, 2.0**51 + 1, 2.0**51 + 0.5, -2.0**51, -2.0**51 - 1,
                      -2.0**51 - 0.5, 2.0**52, -2.0**52, 2.0**52 - 1, 0.49, -0.49, 0.0, 2.0**31])
    c = np.concatenate([c, edges])
    low, dist, hy = _torus_of_chk(c)
    want = (np.vectorize(lambda v: int(np.rint(v)) % 2**32)(c)).astype(np.uint32)
    flagged = (dist >= 0.125) | (hy < 0x43300000) | (hy >= 0x43400000)
    assert np.array_equal(low[~flagged], want[~flagged])
    small = np.abs(c) < 2.0**51
    assert not flagged[small & (np.abs(c - np.rint(c)) < 0.125)].any()
    assert flagged[(c == -2.0**51 - 1) | (c == 2.0**51 + 1) | (c == 2.0**52)].all()   # the high-word checks


def _torus_of_qchk(c):
    """numpy restatement of csrc/fft_wave.h torus_of_qchk (the default kernel's rounding, IEEE
    double): returns (rint(c) mod 2^32 as the kernel extracts it — mantissa bits 2..33 of
    y = c + 1.5 * 2^50 —, round(4c) mod 4 = the low two bits, the high word of y)."""
    c = np.asarray(c, dtype=np.float64)
    y = c + np.float64(1.5 * 2.0**50)
    bits = y.view(np.uint64)
    return (((bits >> np.uint64(2)) & np.uint64(0xFFFFFFFF)).astype(np.uint32),
            (bits & np.uint64(3)).astype(np.uint32), (bits >> np.uint64(32)).astype(np.uint32))


def test_quarter_shifter_rounding_exact_or_flagged():
    """The default kernel's rounding (one 1.5 * 2^50 shifter, ulp 1/4): over the whole product range
    |c| <= 2^52 the extracted word is rint(c) mod 2^32 or the coefficient is flagged (low bits
    != 0: distance >= 1/8; or the high word outside [hi(2^50), hi(2^51)), i.e. |c| >= 2^49); every
    coefficient within 1/8 of an integer and below 2^49 passes, and every one farther than 1/8
    is flagged — the 1/8 rule of DESIGN.md §3.1 on every coefficient."""
    r = np.random.default_rng(11)
    mags = np.concatenate([r.uniform(-2.0**47, 2.0**47, 20000),
                           r.uniform(-2.0**52, 2.0**52, 20000),
                           r.uniform(2.0**48, 2.0**50, 5000) * r.choice([-1, 1], 5000)])
    fr = r.uniform(-0.49, 0.49, mags.shape)
    c = np.floor(mags) + fr
    edges = np.array([2.0**49 - 1, 2.0**49, 2.0**49 + 1, 2.0**49 - 0.5, -2.0**49, -2.0**49 - 1,
                      -2.0**49 + 0.25, 2.0**52, -2.0**52, 0.49, -0.49, 0.124, -0.124, 0.126, 0.0,
                      7.875, 7.87, 2.0**31, -2.0**31 - 0.3])
    c = np.concatenate([c, edges])
    low, q4, hy = _torus_of_qchk(c)
    want = (np.vectorize(lambda v: int(np.rint(v)) % 2**32)(c)).astype(np.uint32)
    flagged = (q4 != 0) | (hy < 0x43100000) | (hy >= 0x43200000)
    assert np.array_equal(low[~flagged], want[~flagged])
    small = np.abs(c) < 2.0**49
    dist = np.abs(c - np.rint(c))
    assert not flagged[small & (dist < 0.125)].any()
    assert flagged[small & (dist > 0.125)].all()
    assert flagged[np.abs(c) > 2.0**49].all()                     # the high-word checks
    assert flagged.sum() > 5000 and (~flagged).sum() > 5000


def _adversarial_keys(shape, rng):
    return {
        # random magnitudes in (2^31 - 2^16, 2^31), all positive
        "allpos16": ((2**31 - 1) - rng.integers(0, 2**16, size=shape, dtype=np.int64)).astype(np.int32),
        # a random high-magnitude constant and a random sign per polynomial
        "polyconst": np.broadcast_to(rng.choice([-1, 1], size=shape[:-1] + (1,)) *
                                     rng.integers(2**31 - 2**24, 2**31, size=shape[:-1] + (1,)),
                                     shape).astype(np.int32),
    }


def _raw_fp64_woks(c, x_a, x_b):
    """The woKS bootstrap through the raw fp64 CMux steps (tfhe_amd_blind_rotate_dev: the v6 step
    kernel with no exactness guard — the library's only unguarded entry, a kernel-test API) and the
    sample extraction in numpy: what the fp64 kernel computes when nothing checks its rounding.
    ACC = (0, X^{2N - barb} (mu, ..., mu)) (lwe-bootstrapping-functions-fft.cu:1427-1431), 500 steps
    with bara_i = modSwitchFromTorus32(x_a[i], 2N), u.a[j] = -acc_a[N - j], u.b = acc_b[0] (lwe.cu:41-56)."""
    import torch
    B = x_a.shape[0]
    acc = np.zeros((B, 2, 1024), np.int32)
    bara = np.zeros((B, 500), np.int32)
    tv = np.full(1024, T.MU, np.int32)
    for k in range(B):
        acc[k, 1] = O.mul_by_xai(2048 - O.modswitch_from(int(x_b[k]), 2048), tv)
        bara[k] = [O.modswitch_from(int(v), 2048) for v in x_a[k]]
    d_acc = torch.from_numpy(acc).cuda()
    c.blind_rotate_dev(d_acc, torch.from_numpy(bara).cuda(), 500)
    c.sync()
    r = d_acc.cpu().numpy().astype(np.int64)
    u_a = np.concatenate([r[:, 0, :1], -r[:, 0, :0:-1]], axis=1)
    return O.i32(u_a), O.i32(r[:, 1, 0])


@pytest.mark.gpu
def test_guard_random_adversarial_keys(keyset):
    """Random high-magnitude keys (not constant: random magnitudes near 2^31, or a random constant
    and sign per polynomial) push the fp64 FFT error across 1/2 on some ciphertexts: through the
    raw, unguarded fp64 steps some of the 64 woKS outputs differ from the exact oracle; through the
    product's woKS call (guarded; the guard cannot be turned off) the guard flags them and every
    output equals the oracle."""
    rng = np.random.default_rng(31)
    keys = _adversarial_keys(keyset.bk.shape, rng)
    B = 64
    x_a = rng.integers(-2**31, 2**31, (B, 500), dtype=np.int64).astype(np.int32)
    x_b = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
    report = {}
    for name, bk in keys.items():
        c = T.Context(bk, keyset.ksk, device=0)
        try:
            g = c.woks_host(T.MU, x_a, x_b)
            d, redo = c.guard_stats()
            u = _raw_fp64_woks(c, x_a, x_b)
        finally:
            c.close()
        want = O.OracleKey(bk, keyset.ksk, use_ntt=True).woks_batch(T.MU, x_a, x_b, nthreads=8)
        wrong = lambda r: int(np.sum(np.any(r[0] != want[0], axis=1) | (r[1] != want[1])))
        report[name] = {"guard_distance": d, "recomputed": redo, "wrong_unguarded": wrong(u),
                        "wrong_guarded": wrong(g)}
    print(report)
    for name, r in report.items():
        assert r["wrong_guarded"] == 0, (name, r)
        assert r["recomputed"] >= r["wrong_unguarded"], (name, r)
        assert r["guard_distance"] >= 0.125, (name, r)
    assert sum(r["wrong_unguarded"] for r in report.values()) > 0, report   # the errors do cross 1/2


def test_guard_threshold_can_only_tighten():
    """tfhe_amd_set_guard_threshold accepts 0 .. 1/8 and refuses anything looser: no call turns the
    exactness guard off."""
    for bad in (0.1251, 0.5, 1.0, -0.1, float("nan")):
        with pytest.raises(T.TfheAmdError):
            T.set_guard_threshold(bad)
    T.set_guard_threshold(0.0)
    T.set_guard_threshold(0.125)
