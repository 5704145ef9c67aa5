"""The oracle pinned against the reference's own compiled sources (CPU, no GPU).

tests/golden/ref_leaf_vectors.npz was produced by tests/golden/make_golden.py from
oracle/_ref/libtfheref.so, i.e. from the reference's gpuParallel/{multiplication,
numeric-functions,lwe-functions,...}.cu compiled in place (oracle/build_ref.sh).
"""
import os

import numpy as np
import pytest

import oracle_ctypes as O

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "ref_leaf_vectors.npz"))


def test_golden_karatsuba_equals_naive():
    # the reference's two exact products agree with each other (fixture sanity)
    assert np.array_equal(G["mul_naive"], G["mul_karatsuba"])


@pytest.mark.parametrize("ntt", [False, True])
def test_negacyclic_product_matches_reference(ntt):
    """multiplication.cu:72-77 torusPolynomialMultNaive == oracle schoolbook and CRT-NTT."""
    z = np.zeros(1024, np.int32)
    for c in range(G["mul_dig"].shape[0]):
        got = O.negacyclic_addmul(z, G["mul_dig"][c], G["mul_poly"][c], ntt=ntt)
        assert np.array_equal(got, G["mul_naive"][c]), c


def test_addmul_matches_reference():
    """multiplication.cu:144-160 torusPolynomialAddMulRKaratsuba (accumulating form)."""
    for c in range(G["addmul_in"].shape[0]):
        got = O.negacyclic_addmul(G["addmul_in"][c], G["mul_dig"][c], G["mul_poly"][c], ntt=True)
        assert np.array_equal(got, G["addmul_out"][c]), c


@pytest.mark.parametrize("M", [2048, 8, 4, 1024])
def test_modswitch_from_matches_reference(M):
    """numeric-functions.cu:60-66.  The uint64 sum (x << 32) + 2^52 wraps for phases in
    [-2^20, 0), which therefore map to 0: the result never reaches Msize (SURVEY.md §7.3
    expected 2048 there; the reference's own code says 0)."""
    got = np.array([O.modswitch_from(int(x), M) for x in G["ms_x"]], np.int32)
    assert np.array_equal(got, G[f"ms_from_{M}"])
    assert got.max() < M
    if M == 2048:
        edge = G["ms_x"] == -2**20
        assert edge.any() and (got[edge] == 0).all()


def test_modswitch_to_matches_reference():
    got = [O.modswitch_to(int(m), int(M)) for m, M in G["ms_to_pairs"]]
    assert got == list(G["ms_to"])


def test_reference_fixture_has_extreme_products():
    # cases 4/5 saturate the dynamic range: digits +-512 times +-2^31
    assert (G["mul_dig"][4] == -512).all() and (G["mul_poly"][4] == -2**31).all()


def test_decomposition_constants_pinned_to_reference():
    """tgsw.cu:7-29 (compiled in place): h = {2^22, 2^12}, offset = 2149580800, kpl 4, Bg 1024,
    halfBg 512, maskMod 1023 — what the product's public TGswParams carries (tests/callers/
    param_dump.cpp), what the kernels' kDecompOffset / shifts hard-code (csrc/params.h), and what
    the oracle decomposes with: the digits reassemble the sample up to the truncated low bits,
    sum_p d_p h_p = x - ((x + offset) mod h[l-1]) (tgsw-functions.cu:322-351 truncates)."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(HERE), "tests", "callers", "_bin", "param_dump")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "callers")])
    got = json.loads(subprocess.check_output([exe]).decode().strip().splitlines()[-1])
    h, off = [int(v) for v in G["tgsw_h"]], int(G["tgsw_offset"][0])
    kpl, bg, half, mask = (int(v) for v in G["tgsw_kpl_bg_halfbg_maskmod"])
    assert (h, off, kpl, bg, half, mask) == ([1 << 22, 1 << 12], 2149580800, 4, 1024, 512, 1023)
    assert (got["h"], got["offset"], got["kpl"], got["Bg"], got["halfBg"], got["maskMod"]) == (h, off, kpl, bg, half, mask)
    params_h = open(os.path.join(os.path.dirname(HERE), "cpu-gpu-tfhe_amd", "csrc", "params.h")).read()
    assert "kDecompOffset = 512u * ((1u << 22) + (1u << 12))" in params_h and 512 * ((1 << 22) + (1 << 12)) == off
    rng = np.random.default_rng(3)
    x = rng.integers(-2**31, 2**31, 1024, dtype=np.int64).astype(np.int32)
    d = O.decompose(x).astype(np.int64)
    assert d.min() >= -half and d.max() < half
    recon = (d[0] * h[0] + d[1] * h[1]) & 0xFFFFFFFF
    err = (x.astype(np.int64) - recon) % 2**32
    assert np.array_equal(err, (x.astype(np.int64) + off) % h[1])


def test_keyswitch_key_index_pinned_to_reference():
    """lwekeyswitch.cu:3-18 (compiled in place): ks[i][j][h] is row (i t + j) base + h of ks0_raw —
    the [i][j][h][n + 1] layout the oracle's key switch reads, the product's flattening and its
    ks-v4 repack assume, and the product's own LweKeySwitchKey struct reproduces."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(HERE), "tests", "callers", "_bin", "param_dump")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "callers")])
    got = json.loads(subprocess.check_output([exe]).decode().strip().splitlines()[-1])
    ref = G["ksk_index"]
    n, t, base = 1024, 8, 4
    i, j, hh = np.meshgrid(np.arange(n), np.arange(t), np.arange(base), indexing="ij")
    assert np.array_equal(ref, ((i * t + j) * base + hh).reshape(-1))
    assert (got["ks_n"], got["ks_t"], got["ks_base"]) == (n, t, base)
    assert np.array_equal(np.array(got["ksk_index"]), ref)
