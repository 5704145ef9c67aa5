"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference path (oracle/tfhe_oracle.c).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as the
checker / the CPU baseline, never as the product.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")

N, n_lwe = 1024, 500
GATES = {"NAND": 0, "OR": 1, "AND": 2, "XOR": 3, "XNOR": 4, "NOR": 5,
         "ANDNY": 6, "ANDYN": 7, "ORNY": 8, "ORYN": 9, "MUX": 10}

_I32P = ctypes.POINTER(ctypes.c_int32)
_lib = None


def _p(a):
    if a is None:
        return None
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_I32P)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(ORACLE_SO)
        L.orc_modSwitchToTorus32.restype = ctypes.c_int32
        L.orc_modSwitchFromTorus32.restype = ctypes.c_int
        L.orc_key_create.restype = ctypes.c_void_p
        L.orc_key_create.argtypes = [_I32P, _I32P, ctypes.c_int]
        L.orc_key_free.argtypes = [ctypes.c_void_p]
        for f in ("orc_mux_rotate", "orc_external_product", "orc_blind_rotate",
                  "orc_bootstrap_woKS", "orc_keyswitch", "orc_bootstrap", "orc_gate",
                  "orc_gate_batch", "orc_bootstrap_woKS_batch", "orc_keyswitch_batch"):
            getattr(L, f).restype = None
        _lib = L
    return _lib


def i32(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.int64).astype(np.int32))


def modswitch_to(mu, M):
    return int(lib().orc_modSwitchToTorus32(int(mu), int(M)))


def modswitch_from(x, M):
    return int(lib().orc_modSwitchFromTorus32(ctypes.c_int32(int(x)), int(M)))


def negacyclic_addmul(res, dig, poly, ntt=False):
    res = i32(res).copy()
    f = lib().orc_negacyclic_addmul_ntt if ntt else lib().orc_negacyclic_addmul_naive
    f(_p(res), _p(i32(dig)), _p(i32(poly)))
    return res


def mul_by_xai(a, x):
    out = np.zeros(N, np.int32)
    lib().orc_mul_by_xai(_p(out), int(a), _p(i32(x)))
    return out


def mul_by_xai_minus_one(a, x):
    out = np.zeros(N, np.int32)
    lib().orc_mul_by_xai_minus_one(_p(out), int(a), _p(i32(x)))
    return out


def decompose(x):
    out = np.zeros((2, N), np.int32)
    lib().orc_decompose(_p(out), _p(i32(x)))
    return out


class OracleKey:
    """Borrowing handle on (bk [500][4][2][1024], ksk [1024][8][4][501]) int32 arrays."""

    def __init__(self, bk, ksk, use_ntt=True):
        self.bk = None if bk is None else i32(bk)
        self.ksk = None if ksk is None else i32(ksk)
        self.h = lib().orc_key_create(_p(self.bk), _p(self.ksk), int(use_ntt))

    def __del__(self):
        if getattr(self, "h", None):
            try:
                lib().orc_key_free(self.h)
            except TypeError:   # interpreter shutdown: module globals already cleared
                pass
            self.h = None

    # ---- single-sample ops
    def external_product(self, acc, i):
        acc = i32(acc).reshape(2 * N).copy()
        lib().orc_external_product(_p(acc), ctypes.c_void_p(self.h), int(i))
        return acc.reshape(2, N)

    def mux_rotate(self, acc, i, a):
        acc = i32(acc).reshape(2 * N).copy()
        lib().orc_mux_rotate(_p(acc), ctypes.c_void_p(self.h), int(i), int(a))
        return acc.reshape(2, N)

    def bootstrap_woks(self, mu, x_a, x_b):
        out_a = np.zeros(N, np.int32)
        out_b = ctypes.c_int32(0)
        lib().orc_bootstrap_woKS(_p(out_a), ctypes.byref(out_b), ctypes.c_void_p(self.h),
                                 ctypes.c_int32(int(mu)), _p(i32(x_a)), ctypes.c_int32(int(x_b)))
        return out_a, out_b.value

    def keyswitch(self, u_a, u_b):
        r_a = np.zeros(n_lwe, np.int32)
        r_b = ctypes.c_int32(0)
        lib().orc_keyswitch(_p(r_a), ctypes.byref(r_b), ctypes.c_void_p(self.h),
                            _p(i32(u_a)), ctypes.c_int32(int(u_b)))
        return r_a, r_b.value

    # ---- batches (SoA)
    def gate_batch(self, gate, ca_a, ca_b, cb_a, cb_b, cc_a=None, cc_b=None, nthreads=0):
        g = GATES[gate] if isinstance(gate, str) else int(gate)
        ca_a = i32(ca_a); B = ca_a.shape[0]
        r_a = np.zeros((B, n_lwe), np.int32)
        r_b = np.zeros(B, np.int32)
        lib().orc_gate_batch(g, B, _p(r_a), _p(r_b), _p(ca_a), _p(i32(ca_b)),
                             _p(i32(cb_a)), _p(i32(cb_b)),
                             _p(None if cc_a is None else i32(cc_a)),
                             _p(None if cc_b is None else i32(cc_b)),
                             ctypes.c_void_p(self.h), int(nthreads))
        return r_a, r_b

    def woks_batch(self, mu, x_a, x_b, nthreads=0):
        x_a = i32(x_a); B = x_a.shape[0]
        o_a = np.zeros((B, N), np.int32)
        o_b = np.zeros(B, np.int32)
        lib().orc_bootstrap_woKS_batch(B, _p(o_a), _p(o_b), ctypes.c_void_p(self.h),
                                       ctypes.c_int32(int(mu)), _p(x_a), _p(i32(x_b)), int(nthreads))
        return o_a, o_b

    def keyswitch_batch(self, u_a, u_b, nthreads=0):
        u_a = i32(u_a); B = u_a.shape[0]
        r_a = np.zeros((B, n_lwe), np.int32)
        r_b = np.zeros(B, np.int32)
        lib().orc_keyswitch_batch(B, _p(r_a), _p(r_b), ctypes.c_void_p(self.h),
                                  _p(u_a), _p(i32(u_b)), int(nthreads))
        return r_a, r_b


def max_threads():
    return int(lib().orc_max_threads())


# --------------------------------------------------------------------- optimized CPU baseline
CPUFFT_SO = os.path.join(ORACLE_DIR, "libcpufft.so")
_fft = None


def fftlib():
    global _fft
    if _fft is None:
        if not os.path.exists(CPUFFT_SO):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(CPUFFT_SO)
        L.cpufft_key_create.restype = ctypes.c_void_p
        L.cpufft_key_create.argtypes = [_I32P, _I32P]
        L.cpufft_key_free.argtypes = [ctypes.c_void_p]
        L.cpufft_max_round_error.restype = ctypes.c_double
        L.cpufft_max_round_error.argtypes = [ctypes.c_void_p]
        L.cpufft_gate_batch.restype = None
        L.cpufft_gate_batch.argtypes = [ctypes.c_int, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32] + [_I32P] * 6 \
            + [ctypes.c_void_p, ctypes.c_int]
        L.cpufft_woks_batch.restype = None
        L.cpufft_woks_batch.argtypes = [ctypes.c_int, _I32P, _I32P, ctypes.c_void_p, ctypes.c_int32, _I32P, _I32P,
                                        ctypes.c_int]
        _fft = L
    return _fft


# gate prologue constants (boot-gates.cu:98-397), as the product's gate_spec
GATE_SPEC = {"NAND": (1 << 29, -1, -1), "OR": (1 << 29, 1, 1), "AND": (-(1 << 29), 1, 1),
             "XOR": (1 << 30, 2, 2), "XNOR": (-(1 << 30), -2, -2), "NOR": (-(1 << 29), -1, -1),
             "ANDNY": (-(1 << 29), -1, 1), "ANDYN": (-(1 << 29), 1, -1), "ORNY": (1 << 29, -1, 1),
             "ORYN": (1 << 29, 1, -1)}


class CpuFftKey:
    """The optimized CPU baseline engine (oracle/cpu_fft.c): fp64 FFT external product,
    OpenMP over gates.  Borrows ksk."""

    def __init__(self, bk, ksk):
        self.bk = i32(bk)
        self.ksk = i32(ksk)
        self.h = fftlib().cpufft_key_create(_p(self.bk), _p(self.ksk))

    def __del__(self):
        if getattr(self, "h", None):
            fftlib().cpufft_key_free(self.h)
            self.h = None

    def max_round_error(self):
        return fftlib().cpufft_max_round_error(self.h)

    def gate_batch(self, gate, ca_a, ca_b, cb_a, cb_b, nthreads=0):
        c, sa, sb = GATE_SPEC[gate]
        ca_a = i32(ca_a); B = ca_a.shape[0]
        r_a = np.zeros((B, n_lwe), np.int32)
        r_b = np.zeros(B, np.int32)
        fftlib().cpufft_gate_batch(B, c, sa, sb, _p(r_a), _p(r_b), _p(ca_a), _p(i32(ca_b)), _p(i32(cb_a)),
                                   _p(i32(cb_b)), self.h, int(nthreads))
        return r_a, r_b

    def woks_batch(self, mu, x_a, x_b, nthreads=0):
        x_a = i32(x_a); B = x_a.shape[0]
        o_a = np.zeros((B, N), np.int32)
        o_b = np.zeros(B, np.int32)
        fftlib().cpufft_woks_batch(B, _p(o_a), _p(o_b), self.h, int(mu), _p(x_a), _p(i32(x_b)), int(nthreads))
        return o_a, o_b
