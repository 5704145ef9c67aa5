"""The v6 blind rotation's fp64 FFT external product, checked on the CPU through
scripts/emu_v6.py — a numpy emulation of the kernel's exact data flow: twiddle tree, the three
radix-8 register passes and their layouts, the DIT inverse on the bit-reversed output and the
post-twist.  The GPU kernel itself is compared with the exact-NTT kernels and the oracle in
tests/test_gpu_parity.py (-m gpu)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
import emu_v6 as E  # noqa: E402


def test_twiddle_tree_roots_and_order():
    W, roots = E.twiddles_v6()
    # stage s has 2^s blocks; odd blocks are i x their even sibling (only even ones stored)
    for s, ws in enumerate(W):
        assert len(ws) == 2 ** s
        for b in range(1, len(ws), 2):
            assert (ws[b] - ws[b - 1]) % E.M == 2048
    # forward slot n evaluates at zeta omega^brv9(n): the DIT inverse relies on this order
    brv = [int(format(n, "09b")[::-1], 2) for n in range(512)]
    assert roots == [(16 * brv[n] + 4) % E.M for n in range(512)]


def _exact(d, bk):
    return sum(E.negacyclic(d[p], bk[p]) for p in range(len(d)))


def test_external_product_exact_with_margin(rng):
    T = E.tables()
    d = rng.integers(-512, 512, (4, 1024))
    bk = rng.integers(-2**31, 2**31, (4, 1024))
    acc = sum(E.fwd(d[p].astype(float), T) * (E.fwd(bk[p].astype(float), T) / 512) for p in range(4))
    want = _exact(d, bk)
    for inv in (E.inv, E.inv_dit):
        c = inv(acc) if inv is E.inv_dit else inv(acc, T)
        assert all(int(g) == int(w) for g, w in zip(np.rint(c).astype(np.int64), want))
        assert np.max(np.abs(c - np.rint(c))) < 0.125          # rounding margin (1/2 needed)


def test_saturated_digits_stay_exact():
    """Extreme but valid inputs: every digit -512 against random keys (the largest |c| the
    decomposition can produce for a given key), and alternating extremes."""
    T = E.tables()
    r = np.random.default_rng(11)
    bk = r.integers(-2**31, 2**31, (4, 1024))
    for d in (np.full((4, 1024), -512), np.where(np.arange(1024) % 2 == 0, 511, -512)[None, :].repeat(4, 0)):
        acc = sum(E.fwd(d[p].astype(float), T) * (E.fwd(bk[p].astype(float), T) / 512) for p in range(4))
        c = E.inv_dit(acc)
        want = _exact(d, bk)
        assert all(int(g) == int(w) for g, w in zip(np.rint(c).astype(np.int64), want))


def test_p3_distance_to_truncating_fft(rng):
    """SURVEY.md §8(c) P3 (diagnostic): the reference's FFTW path converts back with
    Torus32(int64_t(x / N * 2^32)) (fft_processor_fftw.cu:177), i.e. it TRUNCATES the double
    result instead of rounding it.  Emulated on the same transform, that mode differs from the
    exact product (which the engine returns, P1) by exactly 1 on about half of the
    coefficients and never by more."""
    T = E.tables()
    d = rng.integers(-512, 512, (4, 1024))
    bk = rng.integers(-2**31, 2**31, (4, 1024))
    acc = sum(E.fwd(d[p].astype(float), T) * (E.fwd(bk[p].astype(float), T) / 512) for p in range(4))
    c = E.inv_dit(acc)
    exact = np.array([int(x) for x in _exact(d, bk)], dtype=np.int64)
    trunc = np.trunc(c).astype(np.int64)
    delta = np.abs(trunc - exact)
    frac = float(np.mean(delta != 0))
    print(f"P3: truncating-FFT mode differs from the exact product on {frac:.1%} of coefficients "
          f"(max |delta| = {int(delta.max())})")
    assert delta.max() <= 1 and 0.3 < frac < 0.7


def _rotate_rreg(acc, a):
    """numpy restatement of rotate_v6<RREG = true> (blind_rotate_v6.hip): lane L, register r holds
    coefficient L + 64 r; ds_bpermute from lane (L - s) mod 64, then the uniform register rotation
    by q in the negacyclic ring of 32 registers, then lanes L < s take one register further."""
    aa = a & 2047
    s, q = aa & 63, aa >> 6
    reg = acc.reshape(16, 64).astype(np.uint32)          # [r][L]
    V = reg[:, (np.arange(64) - s) % 64]                 # bpermute: V[r][L] = reg[r][(L - s) mod 64]
    ring = np.concatenate([V, (0 - V.astype(np.int64)).astype(np.uint32)])   # 32 registers
    Vq = ring[(np.arange(16) - q) % 32]                  # V[r] = ring[r - q]
    prev = np.concatenate([(0 - Vq[15:16].astype(np.int64)).astype(np.uint32), Vq[:15]])   # V[r - 1]
    lo = np.arange(64) < s
    out = np.where(lo[None, :], prev, Vq)
    return out.reshape(-1)                               # index r * 64 + L = coefficient L + 64 r


def _rotate_rsw_fold(acc, a):
    """numpy restatement of the throughput kernels' form (cmux_v6 RSW, round 6): the permutation
    case q writes each digit source straight from the bpermuted registers V through ring(k)
    (k in [-32, 16): V[k], its negation for k < 0, V[k + 32] below -16), lanes L < s taking
    ring(r - 1 - q) and, for r = 0, -ring(15 - q)."""
    aa = a & 2047
    s, q = aa & 63, aa >> 6
    reg = acc.reshape(16, 64).astype(np.int64)
    V = reg[:, (np.arange(64) - s) % 64]

    def ring(k):
        return V[k] if k >= 0 else (-V[k + 16] if k >= -16 else V[k + 32])
    lo = np.arange(64) < s
    out = np.stack([np.where(lo, ring(r - 1 - q) if r else -ring(15 - q), ring(r - q)) for r in range(16)])
    return (out & 0xFFFFFFFF).astype(np.uint32).reshape(-1)


def test_register_rotation_equals_negacyclic_rotation(rng):
    """The register rotation gives X^a ACC (negacyclic, mod 2^32) for every a the kernel can see,
    including 0, multiples of 64 and the wrap through 1024 and 2048 — the staged form (paired
    kernel) and the throughput kernels' permutation switch with the lane select folded in."""
    acc = rng.integers(0, 2**32, 1024, dtype=np.uint64).astype(np.uint32)
    ext = np.concatenate([acc, (0 - acc.astype(np.int64)).astype(np.uint32)])    # E[k], k < 2N
    for a in list(range(0, 130)) + [511, 512, 513, 960, 1023, 1024, 1025, 1087, 1088, 1984, 2047, 2048] + \
            list(rng.integers(0, 2049, 64)):
        want = ext[(np.arange(1024) - a) % 2048]        # (X^a ACC)[j] = E[(j - a) mod 2N]
        assert np.array_equal(_rotate_rreg(acc, int(a)), want), a
    for a in range(2049):                                # every case of the permutation switch
        want = ext[(np.arange(1024) - a) % 2048]
        assert np.array_equal(_rotate_rsw_fold(acc, a), want), a


def test_four_wave_half_transforms_emulation():
    """The four-wave latency design of round 6 (scripts/emu_v12.py; built as blind_rotate_v12.hip, exact
    on the GPU, measured 2.6 % slower than v6 at B = 1 and removed: DESIGN.md §5.6, profiles/r06_v12_*):
    stage 0 split into halves,
    four radix-4 passes per half over layouts A' B' C' D', the key read at v6's layout, the DIT
    inverse inside each half with the lane factor folded into pass A', stage 8 across the halves:
    v6's spectrum slot for slot and the exact negacyclic product."""
    import emu_v12
    emu_v12.main()


def test_four_wave_lds_slot_maps_conflict_free():
    """The slot maps of the four-wave design's transposes (sAB, sBC, sCD): every 16-B store (8-lane
    groups, 128-B rows) and 16-B load (the four 16-lane groups of ds_read_b128, 256-B rows) of every
    transpose they serve hits distinct banks (MI355X_MICROARCH.md §LDS), and each map is one to one
    within its buffer."""
    lay = {"A": lambda l, r: l + 64 * r, "B": lambda l, r: (l & 15) + 16 * r + 64 * (l >> 4),
           "C": lambda l, r: (l & 3) + 4 * r + 16 * (l >> 2), "D": lambda l, r: 4 * l + r}
    sAB = lambda m: m
    sBC = lambda m: m ^ (((m >> 4) & 3) << 2)
    sCD = lambda m: m + (m >> 2)
    wg = [list(range(8 * k, 8 * k + 8)) for k in range(8)]
    g = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27], [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
    rg = g + [[x + 32 for x in grp] for grp in g]
    uses = [(sAB, "A", "B"), (sAB, "B", "A"), (sBC, "B", "C"), (sBC, "C", "B"), (sCD, "C", "D"), (sCD, "D", "C"),
            (sCD, "D", "D"), (sAB, "A", "A")]
    for f, X, Y in uses:
        assert len({f(m) for m in range(256)}) == 256 and max(f(m) for m in range(256)) < 320
        for r in range(4):
            for grp in wg:
                assert len({f(lay[X](l, r)) % 8 for l in grp}) == 8, (X, Y, r)
            for grp in rg:
                assert len({f(lay[Y](l, r)) % 16 for l in grp}) == 16, (X, Y, r)
