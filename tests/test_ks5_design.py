"""The int8-MFMA key switch (ks-v5, keyswitch.hip) checked on the CPU: a numpy restatement of its
data flow — the balanced signed-byte split of the key (k_ksk_to_v5), the one-hot A fragments
from the 2-digit (nibble) table, the lane maps of v_mfma_i32_32x32x32_i8 (lane l = 32 h + r holds
A[r][16 h + j] and B[16 h + j][r] in byte j; checked on the GPU by scripts/mfma_i8_map.hip), the
int32 sums per limb and their recombination mod 2^32 — against the oracle's key switch
(lwe-keyswitch-functions.cu:101-127).  The GPU kernel itself is compared with the oracle in
tests/test_gpu_parity.py (-m gpu)."""
import numpy as np

from oracle_ctypes import OracleKey

N, T, BASE, NL = 1024, 8, 4, 500
PREC = 1 << 15


def balanced_bytes(w):
    """w (uint32) -> 4 signed bytes s_b, sum s_b 2^(8 b) = w mod 2^32 (k_ksk_to_v5)."""
    v = w.astype(np.uint64)
    out = []
    for _ in range(4):
        s = (v & 0xFF).astype(np.int64)
        s = np.where(s >= 128, s - 256, s)
        out.append(s)
        v = ((v - (s.astype(np.int64) & 0xFFFFFFFF).astype(np.uint64)) & 0xFFFFFFFF) >> 8
    return out


def b_matrix(ksk):
    """K x N int8 matrix in the kernel's order: k = 32 i + 16 h + 4 t + hh (digit j = 4 h + t,
    value hh), n = 32 nb + r with column nb * 8 + r // 4 and limb r % 4 (k_ksk_to_v5's fragment
    bytes, read through the MFMA's B lane map)."""
    cols = 512
    W = np.zeros((N, T, BASE, cols), np.uint32)
    W[:, :, 1:, :NL + 1] = ksk[:, :, 1:, :].astype(np.uint32)      # h = 0: the zero row
    limbs = balanced_bytes(W)                                       # 4 x [i][j][hh][col]
    Bm = np.zeros((N, T, BASE, cols, 4), np.int64)
    for b in range(4):
        Bm[..., b] = limbs[b]
    # k = 32 i + 4 j + hh (= 16 h + 4 t + hh for j = 4 h + t); n = 4 col + limb
    return Bm.reshape(N * T * BASE, cols * 4)


def a_matrix(u_a):
    """one-hot rows: A[m][32 i + 4 j + hh] = [digit j of u_i + 2^15 = hh], built the kernel's
    way — one byte x per (i, lane half h), each nibble of it (2 digits) one table entry of two
    dwords, dword t of the fragment = 1 << (8 a_t)."""
    M = u_a.shape[0]
    u = (u_a.astype(np.int64) + PREC) & 0xFFFFFFFF
    A = np.zeros((M, N, 2, 4, BASE), np.int64)
    nib = np.zeros((16, 2, BASE), np.int64)          # the kernel's lut[n]: (1 << 8 (n >> 2), 1 << 8 (n & 3))
    for n in range(16):
        nib[n, 0, (n >> 2) & 3] = 1
        nib[n, 1, n & 3] = 1
    lut = np.concatenate([nib[np.arange(256) >> 4], nib[np.arange(256) & 15]], axis=1)   # [x][t][hh]
    for h in range(2):
        x = (u >> (24 - 8 * h)) & 255
        A[:, :, h] = lut[x]
    return A.reshape(M, N * T * BASE)


def keyswitch_v5(ksk, u_a, u_b):
    S = a_matrix(u_a).astype(np.float64) @ b_matrix(ksk).astype(np.float64)   # exact: |S| <= 2^20
    S = np.rint(S).astype(np.int64).reshape(u_a.shape[0], 512, 4)
    tot = np.zeros(S.shape[:2], np.int64)
    for b in range(4):
        tot = (tot + (S[:, :, b] << (8 * b))) & 0xFFFFFFFF
    res_a = ((-tot[:, :NL]) & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
    res_b = ((u_b.astype(np.int64) - tot[:, NL]) & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
    return res_a, res_b


def test_balanced_bytes_roundtrip(rng):
    w = rng.integers(0, 2**32, 10000, dtype=np.uint64).astype(np.uint32)
    w[:6] = [0, 1, 0x7F, 0x80, 0xFFFFFFFF, 0x80808080]
    s = balanced_bytes(w)
    assert all(((x >= -128) & (x <= 127)).all() for x in s)
    back = sum(x * (1 << (8 * b)) for b, x in enumerate(s)) & 0xFFFFFFFF
    assert np.array_equal(back.astype(np.uint32), w)


def test_ks5_dataflow_equals_oracle_keyswitch(rng):
    ksk = rng.integers(-2**31, 2**31, (N, T, BASE, NL + 1), dtype=np.int64).astype(np.int32)
    ksk[:, :, 0, :] = 0
    B = 6
    u_a = rng.integers(-2**31, 2**31, (B, N), dtype=np.int64).astype(np.int32)
    u_a[0] = -PREC                      # every digit 0 after the offset: only the b term
    u_a[1] = 2**31 - 1 - PREC           # every digit 3
    u_b = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
    r_a, r_b = keyswitch_v5(ksk, u_a, u_b)
    o_a, o_b = OracleKey(None, ksk).keyswitch_batch(u_a, u_b)
    assert np.array_equal(r_a, o_a) and np.array_equal(r_b, o_b)
