"""The L1 entry points of the reference's TFHE API (north star: `tfhe_blindRotate_FFT` →
`tGswFFTExternMulToTLwe`): gpuParallel/tfhe.h:42-43 (lwe-bootstrapping-functions-fft.cu:676-737,
1408-1456) and tgsw_functions.h:70 (tgsw-fft-operations.cu:124-264), called through the C ABI
exactly as a reference caller would — TLweSample / TorusPolynomial from the library's
allocators, the key's TGswSampleFFT array reached through bk->bkFFT->bkFFT — and compared Torus32
for Torus32 with the exact CPU oracle (orc_external_product / orc_blind_rotate, test-only).
CPU: the TGswSampleFFT layout and the handles' pointer arithmetic; GPU: the products."""
import ctypes

import numpy as np
import pytest

import oracle_ctypes as O
import tfhe_amd as T

N, n = 1024, 500
L = T.lib
_VP = ctypes.c_void_p


class TorusPolynomial(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int), ("coefsT", ctypes.POINTER(ctypes.c_int32))]


class TLweSample(ctypes.Structure):
    _fields_ = [("a", ctypes.POINTER(TorusPolynomial)), ("b", ctypes.POINTER(TorusPolynomial)),
                ("current_variance", ctypes.c_double), ("k", ctypes.c_int)]


class TGswSampleFFT(ctypes.Structure):   # tgsw.h:78-96
    _fields_ = [("all_samples", _VP), ("sample", _VP), ("k", ctypes.c_int), ("l", ctypes.c_int)]


class LweSample(ctypes.Structure):
    _fields_ = [("a", ctypes.POINTER(ctypes.c_int32)), ("b", ctypes.c_int32), ("current_variance", ctypes.c_double)]


for f, res, args in (("new_TLweSample", _VP, [_VP]), ("delete_TLweSample", None, [_VP]),
                     ("new_TorusPolynomial", _VP, [ctypes.c_int]), ("delete_TorusPolynomial", None, [_VP]),
                     ("new_LweSample", _VP, [_VP]), ("delete_LweSample", None, [_VP]),
                     ("tGswFFTExternMulToTLwe", None, [_VP, _VP, _VP]),
                     ("tfhe_blindRotate_FFT", None, [_VP, _VP, ctypes.POINTER(ctypes.c_int), ctypes.c_int, _VP]),
                     ("tfhe_blindRotateAndExtract_FFT", None,
                      [_VP, _VP, _VP, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int, _VP])):
    getattr(L, f).restype = res
    getattr(L, f).argtypes = args


def _ptr(addr):
    return ctypes.c_void_p.from_address(addr).value


def key_parts(keyset):
    """bkFFT = cloud->bkFFT; (bk_params, accum_params, extract_params, the TGswSampleFFT array)"""
    cloud = keyset.cloud
    bkfft = _ptr(cloud + 2 * 8)          # TFheGateBootstrappingCloudKeySet {params, bk, bkFFT}
    # LweBootstrappingKeyFFT {in_out_params, bk_params, accum_params, extract_params, bkFFT, ks}
    return _ptr(bkfft + 8), _ptr(bkfft + 16), _ptr(bkfft + 24), _ptr(bkfft + 32)


def set_tlwe(t, acc):
    s = ctypes.cast(t, ctypes.POINTER(TLweSample)).contents
    for c in range(2):
        ctypes.memmove(s.a[c].coefsT, np.ascontiguousarray(acc[c], np.int32).ctypes.data, 4 * N)


def get_tlwe(t):
    s = ctypes.cast(t, ctypes.POINTER(TLweSample)).contents
    out = np.zeros((2, N), np.int32)
    for c in range(2):
        ctypes.memmove(out[c].ctypes.data, s.a[c].coefsT, 4 * N)
    assert ctypes.addressof(s.b.contents) == ctypes.addressof(s.a[1])   # b aliases a[k]
    return out, s.current_variance


def test_tgsw_sample_fft_array_layout(keyset):
    """bk->bkFFT->bkFFT is an array of kn TGswSampleFFT in the reference layout (k = 1, l = 2),
    so `bkFFT + i` is the reference's indexing (lwe-bootstrapping-functions-fft.cu:705)."""
    assert ctypes.sizeof(TGswSampleFFT) == 24
    _, _, _, arr = key_parts(keyset)
    g = (TGswSampleFFT * n).from_address(arr)
    assert all(x.k == 1 and x.l == 2 for x in g)


@pytest.mark.gpu
def test_external_product_exact(keyset, okey, rng):
    bkp, accp, _, arr = key_parts(keyset)
    t = L.new_TLweSample(accp)
    try:
        for i in (0, 1, 250, 499):
            acc = rng.integers(-2**31, 2**31, (2, N), dtype=np.int64).astype(np.int32)
            if i == 250:
                acc[:] = np.int32(-2**31)     # saturated digits
            set_tlwe(t, acc)
            ctypes.cast(t, ctypes.POINTER(TLweSample)).contents.current_variance = 3.5
            L.tGswFFTExternMulToTLwe(t, arr + 24 * i, bkp)
            got, var = get_tlwe(t)
            want = okey.external_product(acc, i)
            assert np.array_equal(got, want), f"key {i}"
            assert var == 0.0   # tLweFFTClear (tlwe-fft-operations.cu:273-279)
    finally:
        L.delete_TLweSample(t)


@pytest.mark.gpu
def test_external_product_dev_index_checked_on_device(ctx, okey, rng):
    """tfhe_amd_external_product_dev takes its key indices from device memory: an index outside
    [0, 500) leaves that accumulator unchanged (no read past the key); valid neighbours
    in the same launch still get the exact product."""
    import torch
    idx = np.array([3, -1, 500, 1 << 30, 499], np.int32)
    acc = rng.integers(-2**31, 2**31, (len(idx), 2, N), dtype=np.int64).astype(np.int32)
    d_acc = torch.from_numpy(acc.copy()).cuda()
    d_idx = torch.from_numpy(idx).cuda()
    rc = L.tfhe_amd_external_product_dev(ctx.h, len(idx), ctypes.c_void_p(d_idx.data_ptr()),
                                         ctypes.c_void_p(d_acc.data_ptr()), None)
    assert rc == 0
    ctx.sync()
    got = d_acc.cpu().numpy()
    for b, i in enumerate(idx):
        want = okey.external_product(acc[b], int(i)) if 0 <= i < 500 else acc[b]
        assert np.array_equal(got[b], want), (b, int(i))


@pytest.mark.gpu
def test_blind_rotate_fft_exact(keyset, okey, rng):
    bkp, accp, _, arr = key_parts(keyset)
    t = L.new_TLweSample(accp)
    try:
        for start, cnt in ((0, 37), (123, 9), (490, 10)):
            acc = rng.integers(-2**31, 2**31, (2, N), dtype=np.int64).astype(np.int32)
            bara = rng.integers(0, 2 * N, cnt).astype(np.int32)
            bara[::4] = 0                          # skipped steps (:705)
            bara[1] = 2 * N - 1
            if cnt > 5:
                bara[5] = N
            set_tlwe(t, acc)
            ctypes.cast(t, ctypes.POINTER(TLweSample)).contents.current_variance = 1.25
            b = (ctypes.c_int * cnt)(*[int(x) for x in bara])
            L.tfhe_blindRotate_FFT(t, arr + 24 * start, b, cnt, bkp)
            got, var = get_tlwe(t)
            want = acc.copy()
            for i in range(cnt):
                if bara[i]:
                    want = okey.mux_rotate(want, start + i, int(bara[i]))
            assert np.array_equal(got, want), (start, cnt)
            assert var == 1.25
    finally:
        L.delete_TLweSample(t)


@pytest.mark.gpu
def test_blind_rotate_and_extract_fft_exact(keyset, okey, rng):
    """a general test vector v and barb (incl. 0 and N); the full n = 500 key sweep matches the
    oracle's woKS bootstrap when v is the constant mu (what tfhe_bootstrap_woKS_FFT passes)."""
    bkp, accp, extp, arr = key_parts(keyset)
    v = L.new_TorusPolynomial(N)
    r = L.new_LweSample(extp)
    try:
        vp = ctypes.cast(v, ctypes.POINTER(TorusPolynomial)).contents
        rs = ctypes.cast(r, ctypes.POINTER(LweSample)).contents
        for barb, cnt, const in ((17, 40, False), (0, 12, False), (N, 12, False), (None, n, True)):
            if const:
                x_a = rng.integers(-2**31, 2**31, n).astype(np.int32)
                x_b = int(rng.integers(-2**31, 2**31))
                bara = np.array([O.modswitch_from(int(x), 2 * N) for x in x_a], np.int32)
                barb = O.modswitch_from(x_b, 2 * N)
                vec = np.full(N, 1 << 29, np.int32)
            else:
                bara = rng.integers(0, 2 * N, cnt).astype(np.int32)
                bara[::5] = 0
                vec = rng.integers(-2**31, 2**31, N).astype(np.int32)
            ctypes.memmove(vp.coefsT, vec.ctypes.data, 4 * N)
            rs.current_variance = 0.5
            b = (ctypes.c_int * len(bara))(*[int(x) for x in bara])
            L.tfhe_blindRotateAndExtract_FFT(r, v, arr, int(barb), b, len(bara), bkp)
            got_a = np.ctypeslib.as_array(rs.a, (N,)).copy()
            got_b = rs.b
            if const:
                want_a, want_b = okey.bootstrap_woks(1 << 29, x_a, x_b)
            else:
                acc = np.zeros((2, N), np.int32)
                acc[1] = O.mul_by_xai((2 * N - barb) % (2 * N), vec) if barb else vec
                for i in range(len(bara)):
                    if bara[i]:
                        acc = okey.mux_rotate(acc, i, int(bara[i]))
                want_a = np.concatenate([[acc[0][0]], -acc[0][:0:-1].astype(np.int64)]).astype(np.int32)
                want_b = acc[1][0]
            assert np.array_equal(got_a, want_a) and got_b == want_b, (barb, len(bara))
            assert rs.current_variance == 0.5   # extraction leaves it (lwe.cu:41-56)
    finally:
        L.delete_TorusPolynomial(v)
        L.delete_LweSample(r)
