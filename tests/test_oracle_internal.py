"""Internal consistency of the CPU oracle (restatement) — CPU only."""
import numpy as np
import pytest

import oracle_ctypes as O

N = 1024


def test_ntt_product_equals_schoolbook_random(rng):
    for _ in range(3):
        d = rng.integers(-512, 512, N)
        p = rng.integers(-2**31, 2**31, N)
        r0 = rng.integers(-2**31, 2**31, N)
        assert np.array_equal(O.negacyclic_addmul(r0, d, p, ntt=False),
                              O.negacyclic_addmul(r0, d, p, ntt=True))


def test_mul_by_xai_is_negacyclic_rotation(rng):
    x = O.i32(rng.integers(-2**31, 2**31, N))
    for a in (0, 1, 5, 1023, 1024, 1025, 2047):
        got = O.mul_by_xai(a, x)
        want = np.zeros(N, np.int64)
        for j in range(N):
            k = (j + a) % (2 * N)
            if k < N:
                want[k] = x[j]
            else:
                want[k - N] = -np.int64(x[j])
        assert np.array_equal(got, O.i32(want)), a


def test_mul_by_xai_minus_one_edges(rng):
    x = O.i32(rng.integers(-2**31, 2**31, N))
    assert (O.mul_by_xai_minus_one(0, x) == 0).all()
    assert (O.mul_by_xai_minus_one(2048, x) == 0).all()   # the modSwitch == 2N edge
    for a in (1, 700, 1024, 1500, 2047):
        want = O.i32(O.mul_by_xai(a, x).astype(np.int64) - x.astype(np.int64))
        assert np.array_equal(O.mul_by_xai_minus_one(a, x), want)


def test_decomposition_reconstructs(rng):
    """tgsw-functions.cu:300-413: x = sum_p d_p h_p + r with 0 <= r < 2^(32-20): the offset
    trick truncates (it does not round) the low 12 bits."""
    x = rng.integers(-2**31, 2**31, N)
    d = O.decompose(x).astype(np.int64)
    assert d.min() >= -512 and d.max() <= 511
    rec = (d[0] << 22) + (d[1] << 12)
    err = (x - rec) % 2**32
    assert err.max() < 2**12


def test_zero_decomposes_to_zero():
    assert (O.decompose(np.zeros(N)) == 0).all()


def test_external_product_ntt_equals_schoolbook(keyset, rng):
    """Full tGswFFTExternMulToTLwe restatement: NTT mode == schoolbook mode on one key row."""
    k_ntt = O.OracleKey(keyset.bk, None, use_ntt=True)      # full key: the NTT pre-pass reads all 500
    k_naive = O.OracleKey(keyset.bk, None, use_ntt=False)
    acc = rng.integers(-2**31, 2**31, (2, N))
    assert np.array_equal(k_ntt.external_product(acc, 1), k_naive.external_product(acc, 1))
    assert np.array_equal(k_ntt.mux_rotate(acc, 0, 77), k_naive.mux_rotate(acc, 0, 77))


@pytest.mark.parametrize("gate,f", [("NAND", lambda x, y: 1 - (x & y)), ("XNOR", lambda x, y: 1 - (x ^ y)),
                                    ("ANDNY", lambda x, y: (1 - x) & y), ("ORYN", lambda x, y: x | (1 - y))])
def test_oracle_gate_truth_tables(keyset, okey, rng, gate, f):
    x = np.array([0, 0, 1, 1])
    y = np.array([0, 1, 0, 1])
    a = keyset.encrypt(x, rng)
    b = keyset.encrypt(y, rng)
    r_a, r_b = okey.gate_batch(gate, *a, *b)
    assert np.array_equal(keyset.decrypt(r_a, r_b), f(x, y))


def test_oracle_mux_truth_table(keyset, okey, rng):
    s = np.array([0, 0, 1, 1, 0, 1, 0, 1])
    x = np.array([0, 1, 0, 1, 1, 1, 0, 0])
    y = np.array([1, 0, 1, 0, 1, 1, 0, 0])
    r_a, r_b = okey.gate_batch("MUX", *keyset.encrypt(s, rng), *keyset.encrypt(x, rng), *keyset.encrypt(y, rng))
    assert np.array_equal(keyset.decrypt(r_a, r_b), np.where(s == 1, x, y))


def test_oracle_woks_decrypts_under_extracted_key(keyset, okey, rng):
    """woKS output is an LWE of dimension N under the extracted TLWE key; its phase is +-1/8."""
    x = np.array([0, 1, 1, 0])
    a, b = keyset.encrypt(x, rng)
    # bootsAND-style prologue: (0,-1/8) + a + a  -> phase sign = bit
    xa = O.i32(2 * a.astype(np.int64))
    xb = O.i32(2 * b.astype(np.int64) - (1 << 29))
    u_a, u_b = okey.woks_batch(1 << 29, xa, xb)
    ph = keyset.phase_extracted(u_a, u_b).astype(np.int64)
    want = np.where(x == 1, 1 << 29, -(1 << 29))
    assert np.abs(ph - want).max() < (1 << 26)
