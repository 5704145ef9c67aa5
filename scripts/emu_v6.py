"""emu_v6.py — numpy emulation of the v6 (fp64 FFT) blind-rotation transform, layout by layout.

Checks, before any HIP is written, that the twiddle tables (`twiddles_v6`), the three radix-8
register passes (layouts A -> B -> C), the Gentleman-Sande inverse (C -> B -> A) and the
negacyclic fold z_n = a_n + i a_{n+512} compute the exact negacyclic product mod X^1024 + 1,
and reports the worst distance to the nearest integer (the rounding margin).

    python scripts/emu_v6.py
"""
import numpy as np

M = 8192                      # angles in units of 2 pi / 8192


def twiddles_v6():
    """W[s][b] exponents (units 2pi/M) of the merged-twist CT transform of X^512 - i:
    even blocks take the principal square root of their modulus constant, odd blocks i x
    their even sibling, so only even-block twiddles are stored."""
    C = [2048]                # X^512 - e^{i pi / 2}
    W = []
    for s in range(9):
        ws = []
        for b, c in enumerate(C):
            if b % 2 == 0:
                assert c % 2 == 0
                ws.append(c // 2)
            else:
                ws.append((ws[b - 1] + 2048) % M)
        W.append(ws)
        C = [x for w in ws for x in (w, (w + M // 2) % M)]
    return W, C


def cis(e):
    return np.exp(2j * np.pi * np.asarray(e, dtype=np.float64) / M)


def tables():
    W, roots = twiddles_v6()
    L = np.arange(64)
    tu = cis([W[0][0], W[1][0], W[2][0], W[2][2]])                   # pass A (uniform)
    tB = cis([[W[3][l >> 3], W[4][2 * (l >> 3)], W[5][4 * (l >> 3)], W[5][4 * (l >> 3) + 2]] for l in L])
    tC = cis([[W[6][l], W[7][2 * l], W[8][4 * l], W[8][4 * l + 2]] for l in L])
    return tu, tB, tC, roots


def pass_fwd(x, w):
    """x [64][8] complex, w [64][4]: CT stages at register distance 4, 2, 1."""
    x = x.copy()
    w0, w1, w2a, w2b = (w[:, k] for k in range(4))
    def bf(r0, r1, tw):
        t = tw * x[:, r1]
        x[:, r0], x[:, r1] = x[:, r0] + t, x[:, r0] - t
    for r in range(4):
        bf(r, r + 4, w0)
    for r in (0, 1, 4, 5):
        bf(r, r + 2, w1 if r < 4 else 1j * w1)
    for r, tw in ((0, w2a), (2, 1j * w2a), (4, w2b), (6, 1j * w2b)):
        bf(r, r + 1, tw)
    return x


def pass_inv(x, w):
    x = x.copy()
    w0, w1, w2a, w2b = (w[:, k] for k in range(4))
    def bf(r0, r1, tw):
        u, v = x[:, r0], x[:, r1]
        x[:, r0], x[:, r1] = u + v, (u - v) * np.conj(tw)
    for r, tw in ((0, w2a), (2, 1j * w2a), (4, w2b), (6, 1j * w2b)):
        bf(r, r + 1, tw)
    for r in (0, 1, 4, 5):
        bf(r, r + 2, w1 if r < 4 else 1j * w1)
    for r in range(4):
        bf(r, r + 4, w0)
    return x


L = np.arange(64)[:, None]
R = np.arange(8)[None, :]
IDX_A = L + 64 * R
IDX_B = (L & 7) + 8 * R + 64 * (L >> 3)
IDX_C = 8 * L + R


def relayout(x, src, dst):
    flat = np.empty(512, dtype=complex)
    flat[src] = x
    return flat[dst]


def fwd(a, T):
    tu, tB, tC, _ = T
    z = (a[:512] + 1j * a[512:])[IDX_A]
    z = pass_fwd(z, np.broadcast_to(tu, (64, 4)))
    z = pass_fwd(relayout(z, IDX_A, IDX_B), tB)
    return pass_fwd(relayout(z, IDX_B, IDX_C), tC)              # slot 8L + r


def inv(Z, T):
    tu, tB, tC, _ = T
    z = pass_inv(Z, tC)
    z = pass_inv(relayout(z, IDX_C, IDX_B), tB)
    z = pass_inv(relayout(z, IDX_B, IDX_A), np.broadcast_to(tu, (64, 4)))
    flat = relayout(z, IDX_A, np.arange(512))
    return np.concatenate([flat.real, flat.imag])


def negacyclic(a, b):
    full = np.convolve(a.astype(object), b.astype(object))
    out = np.zeros(1024, dtype=object)
    out[:len(full[:1024])] = full[:1024]
    out[:len(full) - 1024] -= full[1024:]
    return out


def main():
    T = tables()
    roots = T[3]
    # output slot n evaluates at root C[9][n]; all 512 roots of X^512 = i, distinct
    assert len(set(roots)) == 512 and all((r - 4) % 16 == 0 for r in roots)
    rng = np.random.default_rng(3)
    # transform is exactly invertible (up to the 512 scale) and linear
    a = rng.standard_normal(1024)
    assert np.allclose(inv(fwd(a, T), T) / 512, a)
    # evaluation semantics: slot n of fwd(a) = A(root_n), A(X) = sum a_j X^j
    Zs = fwd(a, T)
    flat = np.empty(512, dtype=complex)
    flat[IDX_C] = Zs
    j = np.arange(1024)
    for n in (0, 1, 77, 511):
        assert np.isclose(flat[n], np.sum(a * cis(np.array(roots[n]) * j % M)))
    worst = 0.0
    for t in range(6):
        d = rng.integers(-512, 512, (4, 1024))
        bk = rng.integers(-2**31, 2**31, (4, 1024))
        acc = sum(fwd(d[p].astype(float), T) * (fwd(bk[p].astype(float), T) / 512) for p in range(4))
        c = inv(acc, T)
        want = sum(negacyclic(d[p], bk[p]) for p in range(4))
        got = np.rint(c).astype(np.int64)
        assert all(int(g) == int(w) for g, w in zip(got, want)), t
        worst = max(worst, float(np.max(np.abs(c - np.rint(c)))))
    print(f"emu_v6: layouts, twiddles and negacyclic product exact; worst |c - rint(c)| = {worst:.4f}")


if __name__ == "__main__":
    main()


# ---- v6 inverse as radix-2 DIT on the bit-reversed forward output + psi^-n post-twist
# (the forward's slot n evaluates at zeta omega^brv9(n), zeta = e^{i pi / 1024}, omega = e^{2 pi i / 512})
def inv_tables():
    L = np.arange(64)
    e = lambda j, m: np.exp(-2j * np.pi * j / m)
    c8 = np.exp(-1j * np.pi / 4)
    tB = np.stack([e(L & 7, 16), e(L & 7, 32), e(L & 7, 64), e(L & 7, 64) * c8], axis=1)
    tA = np.stack([e(L, 128), e(L, 256), e(L, 512), e(L, 512) * c8], axis=1)
    post = np.exp(-1j * np.pi * (L[:, None] + 64 * np.arange(8)[None, :]) / 1024)   # [L][r]
    return tB, tA, post


def pass_dit(x, a, b, c, c2):
    x = x.copy()
    def bf(r0, r1, W):
        t = W * x[:, r1]
        x[:, r0], x[:, r1] = x[:, r0] + t, x[:, r0] - t
    for r in (0, 2, 4, 6):
        bf(r, r + 1, a)
    for r, W in ((0, b), (1, -1j * b), (4, b), (5, -1j * b)):
        bf(r, r + 2, W)
    for r, W in ((0, c), (1, c2), (2, -1j * c), (3, -1j * c2)):
        bf(r, r + 4, W)
    return x


def inv_dit(Z, folded=True):
    """folded (the kernel since round 2): the post-twist zeta^-(L + 64 r) split into the lane
    factor zeta^-L, applied to pass A's inputs (u inputs of its first butterflies directly, v
    inputs through its first twiddle a zeta^-L), and the register factor e^{-2 pi i r / 32} on
    its outputs; else the 8-entry post-twist table per lane."""
    tB, tA, post = inv_tables()
    one = np.ones(64)
    z = pass_dit(Z, one, one, one, one * np.exp(-1j * np.pi / 4))
    z = pass_dit(relayout(z, IDX_C, IDX_B), *(tB[:, k] for k in range(4)))
    z = relayout(z, IDX_B, IDX_A)
    if folded:
        sig = np.exp(-1j * np.pi * np.arange(64) / 1024)
        z[:, 0::2] = z[:, 0::2] * sig[:, None]
        z = pass_dit(z, tA[:, 0] * sig, tA[:, 1], tA[:, 2], tA[:, 3])
        z = z * np.exp(-2j * np.pi * np.arange(8) / 32)[None, :]
    else:
        z = pass_dit(z, *(tA[:, k] for k in range(4)))
        z = z * post
    flat = relayout(z, IDX_A, np.arange(512))
    return np.concatenate([flat.real, flat.imag])


def check_dit():
    T = tables()
    rng = np.random.default_rng(5)
    a = rng.standard_normal(1024)
    assert np.allclose(inv_dit(fwd(a, T)) / 512, a)
    d = rng.integers(-512, 512, (4, 1024))
    bk = rng.integers(-2**31, 2**31, (4, 1024))
    acc = sum(fwd(d[p].astype(float), T) * (fwd(bk[p].astype(float), T) / 512) for p in range(4))
    c = inv_dit(acc)
    want = sum(negacyclic(d[p], bk[p]) for p in range(4))
    assert all(int(g) == int(w) for g, w in zip(np.rint(c).astype(np.int64), want))
    print(f"emu_v6: DIT inverse + post-twist exact; worst |c - rint(c)| = {np.max(np.abs(c - np.rint(c))):.4f}")


if __name__ == "__main__":
    check_dit()
