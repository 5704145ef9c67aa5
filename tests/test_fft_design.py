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


def test_register_rotation_equals_negacyclic_rotation(rng):
    """The register rotation gives X^a ACC (negacyclic, mod 2^32) for every a the kernel can see,
    including 0, multiples of 64 and the wrap through 1024 and 2048."""
    acc = rng.integers(0, 2**32, 1024, dtype=np.uint64).astype(np.uint32)
    ext = np.concatenate([acc, (0 - acc.astype(np.int64)).astype(np.uint32)])    # E[k], k < 2N
    for a in list(range(0, 130)) + [511, 512, 513, 960, 1023, 1024, 1025, 1087, 1088, 1984, 2047, 2048] + \
            list(rng.integers(0, 2049, 64)):
        want = ext[(np.arange(1024) - a) % 2048]        # (X^a ACC)[j] = E[(j - a) mod 2N]
        assert np.array_equal(_rotate_rreg(acc, int(a)), want), a
