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
