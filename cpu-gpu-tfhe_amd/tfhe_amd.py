"""Python binding (ctypes) of libtfhe_amd.so — the MI355X TFHE gate-bootstrapping engine.

Thin host-side mirror of the C ABI (include/tfhe/tfhe.h = the TFHE API cpuParallel links,
include/tfhe_amd.h = the batched device API).  It exists for the tests and bench.py; the
product is the C ABI itself.  Importing this module loads lib/libtfhe_amd.so and fails
loudly if it is missing (there is no CPU fallback).

Ciphertext batches are SoA numpy / torch arrays: a int32 [B][500], b int32 [B].
"""
import ctypes
import os

import numpy as np

try:
    # torch bundles its own libamdhip64.so.7 (same soname as /opt/rocm's): load it FIRST so
    # that this process has one HIP runtime, shared by torch tensors and our kernels.
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - the C ABI itself does not need torch
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
# TFHE_AMD_LIB selects an alternative build of the same library (A/B kernel variants)
LIB_PATH = os.environ.get("TFHE_AMD_LIB") or os.path.join(HERE, "lib", "libtfhe_amd.so")

N, n_lwe, KPL, KS_T, KS_BASE = 1024, 500, 4, 8, 4
GATES = {"NAND": 0, "OR": 1, "AND": 2, "XOR": 3, "XNOR": 4, "NOR": 5,
         "ANDNY": 6, "ANDYN": 7, "ORNY": 8, "ORYN": 9, "MUX": 10}
MU = 1 << 29   # modSwitchToTorus32(1, 8)

_I32P = ctypes.POINTER(ctypes.c_int32)
_VP = ctypes.c_void_p


class TfheAmdError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise TfheAmdError(
            f"{LIB_PATH} is missing: build it (python -c 'import __graft_entry__ as g; g.build()' "
            "or make -C cpu-gpu-tfhe_amd). There is no CPU fallback.")
    L = ctypes.CDLL(LIB_PATH)
    L.tfhe_amd_version.restype = ctypes.c_char_p
    L.new_default_gate_bootstrapping_parameters.restype = _VP
    L.new_random_gate_bootstrapping_secret_keyset.restype = _VP
    L.new_random_gate_bootstrapping_secret_keyset.argtypes = [_VP]
    L.delete_gate_bootstrapping_secret_keyset.argtypes = [_VP]
    L.delete_gate_bootstrapping_parameters.argtypes = [_VP]
    L.tfhe_amd_export_bk.argtypes = [_VP, _I32P]
    L.tfhe_amd_export_ksk.argtypes = [_VP, _I32P]
    L.tfhe_amd_export_lwe_key.argtypes = [_VP, _I32P]
    L.tfhe_amd_export_tlwe_key.argtypes = [_VP, _I32P]
    L.tfhe_amd_context_create_raw.argtypes = [_I32P, _I32P, ctypes.c_int, ctypes.POINTER(_VP)]
    L.tfhe_amd_context_create.argtypes = [_VP, ctypes.c_int, ctypes.POINTER(_VP)]
    L.tfhe_amd_context_destroy.argtypes = [_VP]
    L.tfhe_amd_context_stream.restype = _VP
    L.tfhe_amd_context_stream.argtypes = [_VP]
    L.tfhe_amd_sync.argtypes = [_VP]
    L.tfhe_amd_reserve.argtypes = [_VP, ctypes.c_int]
    for f in ("tfhe_amd_gate_batch_dev",):
        getattr(L, f).argtypes = [_VP, ctypes.c_int, ctypes.c_int] + [_VP] * 8 + [_VP]
    L.tfhe_amd_gate_batch_host.argtypes = [_VP, ctypes.c_int, ctypes.c_int] + [_I32P] * 8
    L.tfhe_amd_host_alloc.restype = _VP
    L.tfhe_amd_host_alloc.argtypes = [ctypes.c_size_t]
    L.tfhe_amd_host_free.argtypes = [_VP]
    L.tfhe_amd_host_is_pinned.argtypes = [_VP, ctypes.c_size_t]
    L.tfhe_amd_gate_batch_mixed_host.argtypes = [_VP, ctypes.c_int, ctypes.POINTER(ctypes.c_int)] + [_I32P] * 8
    L.tfhe_amd_bootstrap_woks_batch_dev.argtypes = [_VP, ctypes.c_int, ctypes.c_int32] + [_VP] * 4 + [_VP]
    L.tfhe_amd_bootstrap_batch_dev.argtypes = [_VP, ctypes.c_int, ctypes.c_int32] + [_VP] * 4 + [_VP]
    L.tfhe_amd_keyswitch_batch_dev.argtypes = [_VP, ctypes.c_int] + [_VP] * 4 + [_VP]
    L.tfhe_amd_bootstrap_woks_batch_host.argtypes = [_VP, ctypes.c_int, ctypes.c_int32] + [_I32P] * 4
    L.tfhe_amd_bootstrap_batch_host.argtypes = [_VP, ctypes.c_int, ctypes.c_int32] + [_I32P] * 4
    L.tfhe_amd_keyswitch_batch_host.argtypes = [_VP, ctypes.c_int] + [_I32P] * 4
    L.tfhe_amd_blind_rotate_dev.argtypes = [_VP, ctypes.c_int, ctypes.c_int, _VP, _VP, _VP]
    L.tfhe_amd_external_product_dev.argtypes = [_VP, ctypes.c_int, _VP, _VP, _VP]
    L.tfhe_amd_context_create_replica.argtypes = [_VP, ctypes.c_int, ctypes.POINTER(_VP)]
    L.tfhe_amd_context_key_digest.argtypes = [_VP, ctypes.POINTER(ctypes.c_ulonglong)]
    L.tfhe_amd_profile_enable.argtypes = [_VP, ctypes.c_int]
    L.tfhe_amd_profile_read.argtypes = [_VP, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
    L.tfhe_amd_guard_stats.argtypes = [_VP, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong),
                                       ctypes.c_int]
    L.tfhe_amd_set_guard_threshold.argtypes = [ctypes.c_double]
    L.tfhe_amd_fp64_ceiling.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, _VP, _VP]
    L.tfhe_amd_tier1_lane_count.argtypes = [_VP]
    L.tfhe_amd_last_kernels.argtypes = [_VP, ctypes.c_char_p, ctypes.c_int]
    L.tfhe_amd_context_key_bytes.restype = ctypes.c_longlong
    L.tfhe_amd_context_key_bytes.argtypes = [_VP]
    L.tfhe_amd_multi_create_raw.argtypes = [_I32P, _I32P, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                            ctypes.POINTER(_VP)]
    L.tfhe_amd_multi_create.argtypes = [_VP, ctypes.c_int, ctypes.POINTER(_VP)]
    L.tfhe_amd_multi_destroy.argtypes = [_VP]
    L.tfhe_amd_multi_devices.argtypes = [_VP, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.tfhe_amd_multi_context.restype = _VP
    L.tfhe_amd_multi_context.argtypes = [_VP, ctypes.c_int]
    L.tfhe_amd_multi_gate_batch_host.argtypes = [_VP, ctypes.c_int, ctypes.c_int] + [_I32P] * 8
    L.tfhe_amd_shard_range.argtypes = [ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong)]
    L.tfhe_gpu_init.argtypes = [_VP, ctypes.c_int]
    L.tfhe_gpu_boots_batch.argtypes = [ctypes.c_int] + [_I32P] * 8 + [ctypes.c_int, _VP]
    L.tfhe_random_generator_setSeed.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
    L.modSwitchToTorus32.restype = ctypes.c_int32
    L.modSwitchFromTorus32.restype = ctypes.c_int
    L.lwePhase.restype = ctypes.c_int32
    # tfhe_io.h (FILE* entry points)
    for f in ("export_tfheGateBootstrappingSecretKeySet_toFile", "export_tfheGateBootstrappingCloudKeySet_toFile",
              "export_tfheGateBootstrappingParameterSet_toFile"):
        getattr(L, f).argtypes = [_VP, _VP]
    for f in ("new_tfheGateBootstrappingSecretKeySet_fromFile", "new_tfheGateBootstrappingCloudKeySet_fromFile",
              "new_tfheGateBootstrappingParameterSet_fromFile"):
        getattr(L, f).argtypes = [_VP]
        getattr(L, f).restype = _VP
    L.export_gate_bootstrapping_ciphertext_toFile.argtypes = [_VP, _VP, _VP]
    L.import_gate_bootstrapping_ciphertext_fromFile.argtypes = [_VP, _VP, _VP]
    L.new_gate_bootstrapping_ciphertext_array.argtypes = [ctypes.c_int, _VP]
    L.new_gate_bootstrapping_ciphertext_array.restype = _VP
    L.delete_gate_bootstrapping_ciphertext_array.argtypes = [ctypes.c_int, _VP]
    L.delete_gate_bootstrapping_cloud_keyset.argtypes = [_VP]
    return L


lib = _load()


def version():
    return lib.tfhe_amd_version().decode()


def select_kernel(generation):
    """tfhe_amd_select_kernel: blind-rotation kernel generation (0 = default v6, 4 = exact NTT;
    EXPERIMENTAL=1 builds also 1, 2, 3, 5, 7) for A/B runs and cross-checks."""
    _check(lib.tfhe_amd_select_kernel(int(generation)), "select_kernel")


def available_kernels():
    """The blind-rotation generations this build of the library carries (selection restored)."""
    cur = version().split("br-v")[1].split(" ")[0]
    out = [v for v in range(1, 8) if lib.tfhe_amd_select_kernel(v) == 0]
    lib.tfhe_amd_select_kernel(int(cur) if cur.isdigit() else 0)
    return out


def fp64_ceiling(device=0, waves_per_simd=2, seconds=2.0):
    """tfhe_amd_fp64_ceiling: (TFLOP/s, MHz) of register-operand fp64 FMA chains on every SIMD
    for ~seconds: the fp64 rate the device sustains under its power limit (bench roofline)."""
    tf, mhz = ctypes.c_double(), ctypes.c_double()
    _check(lib.tfhe_amd_fp64_ceiling(int(device), int(waves_per_simd), float(seconds), ctypes.byref(tf),
                                     ctypes.byref(mhz)), "fp64_ceiling")
    return tf.value, mhz.value


def set_guard_threshold(distance):
    """tfhe_amd_set_guard_threshold: rounding distance at which the fp64 kernel's results are
    recomputed by the exact NTT kernel (default 1/8, the loosest allowed; 0 recomputes everything)."""
    _check(lib.tfhe_amd_set_guard_threshold(float(distance)), "set_guard_threshold")


def _p(a):
    if a is None:
        return None
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data_as(_I32P)


def _check(rc, what):
    if rc != 0:
        raise TfheAmdError(f"{what} failed with code {rc}")


def i32(x):
    """int32, C-contiguous view of x: the array itself when it already is one (the host batch paths
    then read the caller's memory directly instead of a fresh copy per call — 2 copies of every
    input, ~0.3 ms per 1 024-gate call), else a copy with the values reduced mod 2^32."""
    a = np.asarray(x)
    if a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]:
        return a
    return np.ascontiguousarray(a.astype(np.int64).astype(np.int32))


class _PinnedBlock:
    """one tfhe_amd_host_alloc buffer, freed when the last array viewing it goes"""

    def __init__(self, nbytes):
        self.ptr = lib.tfhe_amd_host_alloc(max(1, nbytes))
        if not self.ptr:
            raise TfheAmdError(f"tfhe_amd_host_alloc({nbytes}) failed")

    def __del__(self):
        if getattr(self, "ptr", None) and lib is not None:
            lib.tfhe_amd_host_free(self.ptr)
            self.ptr = None


def host_empty(shape, dtype=np.int32):
    """A numpy array in caller-owned pinned host memory (tfhe_amd_host_alloc).  Host batch calls
    whose arrays are all such arrays DMA straight from and into them, with no staging copy."""
    dt = np.dtype(dtype)
    n = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
    blk = _PinnedBlock(n)
    buf = (ctypes.c_char * max(1, n)).from_address(blk.ptr)
    buf._owner = blk
    return np.frombuffer(buf, dtype=dt, count=n // dt.itemsize).reshape(shape)


def host_copy(x, dtype=np.int32):
    """x copied into a new pinned array (host_empty)"""
    a = np.asarray(x)
    out = host_empty(a.shape, dtype)
    out[...] = a
    return out


def is_pinned(a):
    """whether the array's bytes lie inside one tfhe_amd_host_alloc buffer"""
    a = np.asarray(a)
    return bool(lib.tfhe_amd_host_is_pinned(a.ctypes.data, a.nbytes))


# --------------------------------------------------------------------- files (tfhe_io.h)

_libc = ctypes.CDLL(None)
_libc.fopen.restype = _VP
_libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
_libc.fclose.argtypes = [_VP]


class _File:
    """FILE* for the tfhe_io.h entry points (they take C stdio streams, like the reference)."""

    def __init__(self, path, mode):
        self.f = _libc.fopen(os.fsencode(path), mode.encode())
        if not self.f:
            raise OSError(f"cannot open {path} ({mode})")

    def __enter__(self):
        return self.f

    def __exit__(self, *exc):
        _libc.fclose(self.f)


class LweSampleC(ctypes.Structure):
    """struct LweSample (lwesamples.h:18-29)."""
    _fields_ = [("a", _I32P), ("b", ctypes.c_int32), ("current_variance", ctypes.c_double)]


def write_ciphertexts(path, params, a, b, variance=0.0, mode="wb"):
    """export_gate_bootstrapping_ciphertext_toFile for each row of the SoA batch (a [B][n], b [B])."""
    a = i32(a); b = i32(b); B = a.shape[0]
    arr = lib.new_gate_bootstrapping_ciphertext_array(B, params)
    try:
        s = (LweSampleC * B).from_address(arr)
        with _File(path, mode) as f:
            for i in range(B):
                ctypes.memmove(s[i].a, a[i].ctypes.data, 4 * n_lwe)
                s[i].b = int(b[i]); s[i].current_variance = float(variance)
                lib.export_gate_bootstrapping_ciphertext_toFile(f, ctypes.byref(s[i]), params)
    finally:
        lib.delete_gate_bootstrapping_ciphertext_array(B, arr)


def read_ciphertexts(path, params, B):
    """import_gate_bootstrapping_ciphertext_fromFile B times -> (a [B][n], b [B], variance [B])."""
    arr = lib.new_gate_bootstrapping_ciphertext_array(B, params)
    a = np.zeros((B, n_lwe), np.int32); b = np.zeros(B, np.int32); v = np.zeros(B)
    try:
        s = (LweSampleC * B).from_address(arr)
        with _File(path, "rb") as f:
            for i in range(B):
                lib.import_gate_bootstrapping_ciphertext_fromFile(f, ctypes.byref(s[i]), params)
                ctypes.memmove(a[i].ctypes.data, s[i].a, 4 * n_lwe)
                b[i] = s[i].b; v[i] = s[i].current_variance
    finally:
        lib.delete_gate_bootstrapping_ciphertext_array(B, arr)
    return a, b, v


# --------------------------------------------------------------------- keys (host)

class SecretKeyset:
    """new_random_gate_bootstrapping_secret_keyset (tfhe_gate_bootstrapping.cu:57-68) seeded
    through tfhe_random_generator_setSeed; exposes the key material as numpy arrays."""

    def __init__(self, seed=(314, 1592, 657), path=None):
        """seeded keygen, or (path=...) new_tfheGateBootstrappingSecretKeySet_fromFile."""
        if path is None:
            s = (ctypes.c_uint32 * len(seed))(*seed)
            lib.tfhe_random_generator_setSeed(s, len(seed))
            self.own_params = lib.new_default_gate_bootstrapping_parameters(110)
            self.h = lib.new_random_gate_bootstrapping_secret_keyset(self.own_params)
        else:
            self.own_params = None            # belongs to the keyset read from the file
            with _File(path, "rb") as f:
                self.h = lib.new_tfheGateBootstrappingSecretKeySet_fromFile(f)
        if not self.h:
            raise TfheAmdError("keygen failed")
        self.params = ctypes.c_void_p.from_address(self.h).value     # key->params
        self.bk = np.zeros((n_lwe, KPL, 2, N), np.int32)
        self.ksk = np.zeros((N, KS_T, KS_BASE, n_lwe + 1), np.int32)
        self.lwe_key = np.zeros(n_lwe, np.int32)
        _check(lib.tfhe_amd_export_bk(ctypes.c_void_p(self._cloud()), _p(self.bk)), "export_bk")
        _check(lib.tfhe_amd_export_ksk(ctypes.c_void_p(self._cloud()), _p(self.ksk)), "export_ksk")
        _check(lib.tfhe_amd_export_lwe_key(ctypes.c_void_p(self.h), _p(self.lwe_key)), "export_lwe_key")
        self.tlwe_key = np.zeros(N, np.int32)
        _check(lib.tfhe_amd_export_tlwe_key(ctypes.c_void_p(self.h), _p(self.tlwe_key)), "export_tlwe_key")

    def save(self, path):
        """export_tfheGateBootstrappingSecretKeySet_toFile"""
        with _File(path, "wb") as f:
            lib.export_tfheGateBootstrappingSecretKeySet_toFile(f, self.h)

    def save_cloud(self, path):
        """export_tfheGateBootstrappingCloudKeySet_toFile(F, &key->cloud)"""
        with _File(path, "wb") as f:
            lib.export_tfheGateBootstrappingCloudKeySet_toFile(f, self._cloud())

    def _cloud(self):
        # &key->cloud: TFheGateBootstrappingSecretKeySet = {params*, lwe_key*, tgsw_key*, cloud}
        return self.h + 3 * ctypes.sizeof(ctypes.c_void_p)

    @property
    def cloud(self):
        return self._cloud()

    def close(self):
        if self.h:
            lib.delete_gate_bootstrapping_secret_keyset(self.h)
            self.h = None
        if self.own_params:
            lib.delete_gate_bootstrapping_parameters(self.own_params)
            self.own_params = None

    # numpy-side encryption with the same secret (fast path for big batches; the product's
    # bootsSymEncrypt is covered by its own test)
    def encrypt(self, bits, rng, stdev=2.4349504419032758e-05):
        bits = np.asarray(bits).astype(np.int64)
        B = bits.shape[0]
        a = rng.integers(-2**31, 2**31, (B, n_lwe), dtype=np.int64)
        mu = np.where(bits != 0, MU, -MU)
        noise = np.rint(rng.normal(0.0, stdev, B) * 2**32).astype(np.int64)
        b = (a @ self.lwe_key.astype(np.int64) + mu + noise)
        return i32(a), i32(b)

    def phase(self, a, b):
        a = np.asarray(a).astype(np.int64)
        ph = (np.asarray(b).astype(np.int64) - a @ self.lwe_key.astype(np.int64)) & 0xFFFFFFFF
        return ph.astype(np.uint32).view(np.int32)

    def decrypt(self, a, b):
        return (self.phase(a, b) > 0).astype(np.int32)

    def phase_extracted(self, u_a, u_b):
        """phase of a woKS output (dimension N) under the extracted key (tLweExtractKey)."""
        u_a = np.asarray(u_a).astype(np.int64)
        ph = (np.asarray(u_b).astype(np.int64) - u_a @ self.tlwe_key.astype(np.int64)) & 0xFFFFFFFF
        return ph.astype(np.uint32).view(np.int32)


class CloudKeyset:
    """new_tfheGateBootstrappingCloudKeySet_fromFile (tfhe_io.cu:1117): what cloud.cpp loads."""

    def __init__(self, path):
        with _File(path, "rb") as f:
            self.h = lib.new_tfheGateBootstrappingCloudKeySet_fromFile(f)
        if not self.h:
            raise TfheAmdError(f"cannot read cloud key {path}")
        self.params = ctypes.c_void_p.from_address(self.h).value      # bk->params

    def save(self, path):
        with _File(path, "wb") as f:
            lib.export_tfheGateBootstrappingCloudKeySet_toFile(f, self.h)

    def export_bk(self):
        bk = np.zeros((n_lwe, KPL, 2, N), np.int32)
        _check(lib.tfhe_amd_export_bk(ctypes.c_void_p(self.h), _p(bk)), "export_bk")
        return bk

    def export_ksk(self):
        ksk = np.zeros((N, KS_T, KS_BASE, n_lwe + 1), np.int32)
        _check(lib.tfhe_amd_export_ksk(ctypes.c_void_p(self.h), _p(ksk)), "export_ksk")
        return ksk

    def close(self):
        if self.h:
            lib.delete_gate_bootstrapping_cloud_keyset(self.h)
            self.h = None


# --------------------------------------------------------------------- device context

class Context:
    """TfheAmdContext: key material of one cloud key on one GPU (tfhe_amd_context_create_raw)."""

    def __init__(self, bk, ksk, device=0):
        self.bk = i32(bk)
        self.ksk = i32(ksk)
        h = _VP()
        _check(lib.tfhe_amd_context_create_raw(_p(self.bk), _p(self.ksk), int(device), ctypes.byref(h)),
               "tfhe_amd_context_create_raw")
        self.h = h.value
        self.device = device

    @classmethod
    def replica_of(cls, src, device):
        """tfhe_amd_context_create_replica: src's converted device key copied device to device"""
        h = _VP()
        _check(lib.tfhe_amd_context_create_replica(src.h, int(device), ctypes.byref(h)), "context_create_replica")
        c = cls.__new__(cls)
        c.bk, c.ksk, c.h, c.device = src.bk, src.ksk, h.value, device
        return c

    def key_digest(self):
        """FNV-1a 64 of the context's device key bytes (tfhe_amd_context_key_digest)"""
        d = ctypes.c_ulonglong()
        _check(lib.tfhe_amd_context_key_digest(self.h, ctypes.byref(d)), "context_key_digest")
        return d.value

    def close(self):
        if getattr(self, "h", None):
            lib.tfhe_amd_context_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return lib.tfhe_amd_context_stream(self.h)

    def key_bytes(self):
        """device bytes of this context's key material (tfhe_amd_context_key_bytes)"""
        return int(lib.tfhe_amd_context_key_bytes(self.h))

    def sync(self):
        _check(lib.tfhe_amd_sync(self.h), "sync")

    def reserve(self, B):
        _check(lib.tfhe_amd_reserve(self.h, int(B)), "reserve")

    # ---- host (numpy) batches
    def gate_host(self, gate, ca_a, ca_b, cb_a, cb_b, cc_a=None, cc_b=None, out=None):
        """tfhe_amd_gate_batch_host; out = (r_a [B][500], r_b [B]) int32 arrays to reuse (else new ones).
        With every array pinned (host_empty / host_copy) the kernels read the inputs in place and the
        results are copied straight into `out`.  `out` must be C-contiguous: the library writes B x 500
        consecutive words (a strided view would be overwritten past its rows)."""
        g = GATES[gate] if isinstance(gate, str) else int(gate)
        ca_a = i32(ca_a); B = ca_a.shape[0]
        if out is not None:
            r_a, r_b = out
            if r_a.shape != (B, n_lwe) or r_b.shape != (B,) or r_a.dtype != np.int32 or r_b.dtype != np.int32:
                raise TfheAmdError("out: need int32 arrays [B][500] and [B]")
            if not (r_a.flags["C_CONTIGUOUS"] and r_b.flags["C_CONTIGUOUS"]):
                raise TfheAmdError("out: need C-contiguous arrays")
        else:
            r_a = np.zeros((B, n_lwe), np.int32); r_b = np.zeros(B, np.int32)
        _check(lib.tfhe_amd_gate_batch_host(self.h, g, B, _p(r_a), _p(r_b), _p(ca_a), _p(i32(ca_b)),
                                            _p(i32(cb_a)), _p(i32(cb_b)),
                                            _p(None if cc_a is None else i32(cc_a)),
                                            _p(None if cc_b is None else i32(cc_b))), "gate_batch_host")
        return r_a, r_b

    def gate_mixed_host(self, gates, ca_a, ca_b, cb_a, cb_b, cc_a=None, cc_b=None):
        """tfhe_amd_gate_batch_mixed_host: gate i of kind gates[i] (names or codes) on row i, all in
        one blind-rotation and one key-switch launch."""
        g = np.array([GATES[x] if isinstance(x, str) else int(x) for x in gates], dtype=np.int32)
        ca_a = i32(ca_a); B = ca_a.shape[0]
        if g.shape != (B,):
            raise TfheAmdError(f"gates: need one gate kind per row ({B}), got {g.shape[0]}")
        r_a = np.zeros((B, n_lwe), np.int32); r_b = np.zeros(B, np.int32)
        _check(lib.tfhe_amd_gate_batch_mixed_host(self.h, B, g.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _p(r_a),
                                                  _p(r_b), _p(ca_a), _p(i32(ca_b)), _p(i32(cb_a)), _p(i32(cb_b)),
                                                  _p(None if cc_a is None else i32(cc_a)),
                                                  _p(None if cc_b is None else i32(cc_b))), "gate_batch_mixed_host")
        return r_a, r_b

    def woks_host(self, mu, x_a, x_b):
        x_a = i32(x_a); B = x_a.shape[0]
        u_a = np.zeros((B, N), np.int32); u_b = np.zeros(B, np.int32)
        _check(lib.tfhe_amd_bootstrap_woks_batch_host(self.h, B, int(mu), _p(x_a), _p(i32(x_b)), _p(u_a), _p(u_b)),
               "woks_host")
        return u_a, u_b

    def bootstrap_host(self, mu, x_a, x_b):
        x_a = i32(x_a); B = x_a.shape[0]
        r_a = np.zeros((B, n_lwe), np.int32); r_b = np.zeros(B, np.int32)
        _check(lib.tfhe_amd_bootstrap_batch_host(self.h, B, int(mu), _p(x_a), _p(i32(x_b)), _p(r_a), _p(r_b)),
               "bootstrap_host")
        return r_a, r_b

    def keyswitch_host(self, u_a, u_b):
        u_a = i32(u_a); B = u_a.shape[0]
        r_a = np.zeros((B, n_lwe), np.int32); r_b = np.zeros(B, np.int32)
        _check(lib.tfhe_amd_keyswitch_batch_host(self.h, B, _p(u_a), _p(i32(u_b)), _p(r_a), _p(r_b)),
               "keyswitch_host")
        return r_a, r_b

    # ---- device (torch) batches: tensors must be int32 CUDA/HIP tensors, contiguous
    def _dev_check(self, t, shape, name):
        """The kernels index by shape and run on this context's GPU: refuse anything that would
        make them read or write out of bounds, or touch another device's memory, before it
        reaches the GPU."""
        if t is None:
            raise TfheAmdError(f"{name}: missing tensor")
        if not t.is_cuda or t.dtype != torch.int32 or not t.is_contiguous() or tuple(t.shape) != shape:
            raise TfheAmdError(f"{name}: need a contiguous int32 GPU tensor of shape {shape}, got "
                               f"{tuple(t.shape)} {t.dtype} cuda={t.is_cuda} contiguous={t.is_contiguous()}")
        if t.device.index is not None and t.device.index != self.device:
            raise TfheAmdError(f"{name}: tensor is on cuda:{t.device.index}, the context on cuda:{self.device}")

    def gate_dev(self, gate, res_a, res_b, ca_a, ca_b, cb_a, cb_b, cc_a=None, cc_b=None, stream=None):
        g = GATES[gate] if isinstance(gate, str) else int(gate)
        B = ca_a.shape[0]
        named = [("res_a", res_a, (B, n_lwe)), ("res_b", res_b, (B,)), ("ca_a", ca_a, (B, n_lwe)),
                 ("ca_b", ca_b, (B,)), ("cb_a", cb_a, (B, n_lwe)), ("cb_b", cb_b, (B,))]
        if g == GATES["MUX"]:
            named += [("cc_a", cc_a, (B, n_lwe)), ("cc_b", cc_b, (B,))]
        for name, t, shape in named:
            self._dev_check(t, shape, name)
        ptr = (lambda t: None if t is None else t.data_ptr())
        _check(lib.tfhe_amd_gate_batch_dev(self.h, g, B, ptr(res_a), ptr(res_b), ptr(ca_a), ptr(ca_b),
                                           ptr(cb_a), ptr(cb_b), ptr(cc_a), ptr(cc_b), stream),
               "gate_batch_dev")

    def blind_rotate_dev(self, acc, bara, iters, stream=None):
        B = acc.shape[0]
        self._dev_check(acc, (B, 2, 1024), "acc")
        if int(iters) > 0:
            self._dev_check(bara, (B, int(iters)), "bara")
        _check(lib.tfhe_amd_blind_rotate_dev(self.h, B, int(iters), acc.data_ptr(),
                                             None if bara is None else bara.data_ptr(), stream),
               "blind_rotate_dev")

    def guard_stats(self, reset=False):
        """(largest rounding distance measured, ciphertexts recomputed exactly) since the last
        reset (tfhe_amd_guard_stats; synchronizes the device)."""
        d = ctypes.c_double(); r = ctypes.c_longlong()
        _check(lib.tfhe_amd_guard_stats(self.h, ctypes.byref(d), ctypes.byref(r), int(bool(reset))), "guard_stats")
        return d.value, r.value

    def last_kernels(self):
        """tfhe_amd_last_kernels: the kernels (and variants) the last batch call enqueued."""
        buf = ctypes.create_string_buffer(1024)
        n = lib.tfhe_amd_last_kernels(self.h, buf, 1024)
        if n < 0:
            raise TfheAmdError(f"last_kernels failed (rc={n})")
        return [k for k in buf.value.decode().split(",") if k]

    def profile_enable(self, on=True):
        _check(lib.tfhe_amd_profile_enable(self.h, int(on)), "profile_enable")

    def profile_read(self):
        br = ctypes.c_double(); ks = ctypes.c_double(); nb = ctypes.c_int(); nk = ctypes.c_int()
        _check(lib.tfhe_amd_profile_read(self.h, ctypes.byref(br), ctypes.byref(nb), ctypes.byref(ks),
                                         ctypes.byref(nk)), "profile_read")
        return {"br_ms": br.value, "br_launches": nb.value, "ks_ms": ks.value, "ks_launches": nk.value}


# --------------------------------------------------------------------- several GPUs (§8(e))

def shard_range(total, rank, world):
    """tfhe_amd_shard_range: the library's contiguous shard [lo, hi) (= shard.shard_range)."""
    lo, hi = ctypes.c_longlong(), ctypes.c_longlong()
    _check(lib.tfhe_amd_shard_range(int(total), int(rank), int(world), ctypes.byref(lo), ctypes.byref(hi)),
           "shard_range")
    return lo.value, hi.value


class MultiContext:
    """TfheAmdMulti: one key replica and worker thread per device; a batch of independent gates
    is split into contiguous shards, one per device (tfhe_amd_multi_gate_batch_host)."""

    def __init__(self, bk, ksk, devices):
        self.bk = i32(bk)
        self.ksk = i32(ksk)
        self.devices = [int(d) for d in devices]
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        h = _VP()
        _check(lib.tfhe_amd_multi_create_raw(_p(self.bk), _p(self.ksk), arr, len(self.devices), ctypes.byref(h)),
               "tfhe_amd_multi_create_raw")
        self.h = h.value

    def close(self):
        if getattr(self, "h", None):
            lib.tfhe_amd_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def gate_host(self, gate, ca_a, ca_b, cb_a, cb_b, cc_a=None, cc_b=None):
        g = GATES[gate] if isinstance(gate, str) else int(gate)
        ca_a = i32(ca_a); B = ca_a.shape[0]
        r_a = np.zeros((B, n_lwe), np.int32); r_b = np.zeros(B, np.int32)
        _check(lib.tfhe_amd_multi_gate_batch_host(self.h, g, B, _p(r_a), _p(r_b), _p(ca_a), _p(i32(ca_b)),
                                                  _p(i32(cb_a)), _p(i32(cb_b)),
                                                  _p(None if cc_a is None else i32(cc_a)),
                                                  _p(None if cc_b is None else i32(cc_b))), "multi_gate_batch_host")
        return r_a, r_b

    def gate_dev(self, gate, shards, streams=None):
        """tfhe_amd_multi_gate_batch_dev: shards[i] = (res_a, res_b, ca_a, ca_b, cb_a, cb_b[, cc_a, cc_b])
        int32 tensors on slot i's device (the shard of that slot; may be empty).  Enqueued on
        every slot; call sync()."""
        g = GATES[gate] if isinstance(gate, str) else int(gate)
        k = len(self.devices)
        if len(shards) != k:
            raise TfheAmdError(f"need {k} shards, got {len(shards)}")
        counts = (ctypes.c_int * k)()
        arrs = [(_VP * k)() for _ in range(8)]
        for i, sh in enumerate(shards):
            B = sh[2].shape[0]
            counts[i] = B
            shapes = [(B, n_lwe), (B,)] * (4 if g == GATES["MUX"] else 3)
            for j, t in enumerate(sh[:len(shapes)]):
                if not t.is_cuda or t.dtype != torch.int32 or not t.is_contiguous() or tuple(t.shape) != shapes[j]:
                    raise TfheAmdError(f"shard {i} tensor {j}: need a contiguous int32 GPU tensor {shapes[j]}")
                if t.device.index is not None and t.device.index != self.devices[i]:
                    raise TfheAmdError(f"shard {i} tensor {j} is on cuda:{t.device.index}, slot device {self.devices[i]}")
                arrs[j][i] = t.data_ptr()
        st = None
        if streams is not None:
            st = (_VP * k)(*[s for s in streams])
        cc = (arrs[6], arrs[7]) if g == GATES["MUX"] else (None, None)
        _check(lib.tfhe_amd_multi_gate_batch_dev(self.h, g, counts, arrs[0], arrs[1], arrs[2], arrs[3], arrs[4],
                                                 arrs[5], cc[0], cc[1], st), "multi_gate_batch_dev")

    def sync(self):
        _check(lib.tfhe_amd_multi_sync(self.h), "multi_sync")

    def circuit_host(self, circ, B, in_wires, in_a, in_b, out_wires):
        """tfhe_amd_multi_circuit_run_host: the B instances sharded over the devices; in_a [n_in][B][500],
        in_b [n_in][B] for the wires in_wires -> (out_a [n_out][B][500], out_b [n_out][B])."""
        in_a = i32(in_a); in_b = i32(in_b)
        n_in, n_out = len(in_wires), len(out_wires)
        if in_a.shape != (n_in, B, n_lwe) or in_b.shape != (n_in, B):
            raise TfheAmdError(f"inputs: need [{n_in}][{B}][500] / [{n_in}][{B}], got {in_a.shape} / {in_b.shape}")
        out_a = np.zeros((n_out, B, n_lwe), np.int32); out_b = np.zeros((n_out, B), np.int32)
        _check(lib.tfhe_amd_multi_circuit_run_host(self.h, circ.h, int(B), n_in, _ids(in_wires), _p(in_a), _p(in_b),
                                                   n_out, _ids(out_wires), _p(out_a), _p(out_b)),
               "multi_circuit_run_host")
        return out_a, out_b

    def circuit_dev(self, circ, shards, streams=None):
        """tfhe_amd_multi_circuit_run_dev: shards[i] = (wires_a [n_wires][B_i][500], wires_b [n_wires][B_i])
        on slot i's device.  Enqueued on every slot; call sync()."""
        k = len(self.devices)
        if len(shards) != k:
            raise TfheAmdError(f"need {k} shards, got {len(shards)}")
        for i, sh in enumerate(shards):
            wa, wb = sh[0], sh[1]
            if wa.dim() != 3 or wa.shape[2] != n_lwe or tuple(wb.shape) != tuple(wa.shape[:2]):
                raise TfheAmdError(f"shard {i}: need wires_a [n_wires][B][500] and wires_b [n_wires][B], "
                                   f"got {tuple(wa.shape)} / {tuple(wb.shape)}")
            for j, t in enumerate((wa, wb)):
                if not t.is_cuda or t.dtype != torch.int32 or not t.is_contiguous():
                    raise TfheAmdError(f"shard {i} tensor {j}: need a contiguous int32 GPU tensor")
                if t.device.index is not None and t.device.index != self.devices[i]:
                    raise TfheAmdError(f"shard {i} tensor {j} is on cuda:{t.device.index}, slot device {self.devices[i]}")
        counts = (ctypes.c_int * k)(*[int(sh[0].shape[1]) for sh in shards])
        wa = (_VP * k)(*[sh[0].data_ptr() for sh in shards])
        wb = (_VP * k)(*[sh[1].data_ptr() for sh in shards])
        st = None if streams is None else (_VP * k)(*streams)
        _check(lib.tfhe_amd_multi_circuit_run_dev(self.h, circ.h, counts, wa, wb, st), "multi_circuit_run_dev")

    def key_digest(self, i):
        """FNV-1a 64 of slot i's device key bytes (slots > 0 are peer-copied replicas of slot 0)"""
        d = ctypes.c_ulonglong()
        _check(lib.tfhe_amd_context_key_digest(lib.tfhe_amd_multi_context(self.h, int(i)), ctypes.byref(d)),
               "context_key_digest")
        return d.value

    def guard_stats(self, reset=False):
        """per device slot: (largest rounding distance, ciphertexts recomputed exactly)"""
        out = []
        for i in range(len(self.devices)):
            c = lib.tfhe_amd_multi_context(self.h, i)
            d = ctypes.c_double(); r = ctypes.c_longlong()
            _check(lib.tfhe_amd_guard_stats(c, ctypes.byref(d), ctypes.byref(r), int(bool(reset))), "guard_stats")
            out.append((d.value, r.value))
        return out


def gpu_init(cloud, device_mask):
    """tfhe_gpu_init(cloud key, device_mask): register a multi-device context for the key."""
    _check(lib.tfhe_gpu_init(ctypes.c_void_p(cloud), int(device_mask)), "tfhe_gpu_init")


def gpu_boots_batch(cloud, gate, ca_a, ca_b, cb_a, cb_b, cc_a=None, cc_b=None):
    """tfhe_gpu_boots_batch over the key's registered devices (SURVEY.md §8(b) Tier-2)."""
    g = GATES[gate] if isinstance(gate, str) else int(gate)
    ca_a = i32(ca_a); B = ca_a.shape[0]
    r_a = np.zeros((B, n_lwe), np.int32); r_b = np.zeros(B, np.int32)
    _check(lib.tfhe_gpu_boots_batch(g, _p(r_a), _p(r_b), _p(ca_a), _p(i32(ca_b)), _p(i32(cb_a)), _p(i32(cb_b)),
                                    _p(None if cc_a is None else i32(cc_a)), _p(None if cc_b is None else i32(cc_b)),
                                    B, ctypes.c_void_p(cloud)), "tfhe_gpu_boots_batch")
    return r_a, r_b


# --------------------------------------------------------------------- circuits (§8(f) row 1)

GATES.update({"MAJ": 11, "XOR3": 12, "NOT": 13, "COPY": 14, "CONST": 15})
_IP = ctypes.POINTER(ctypes.c_int)
lib.tfhe_amd_circuit_create.argtypes = [ctypes.POINTER(_VP)]
lib.tfhe_amd_circuit_destroy.argtypes = [_VP]
lib.tfhe_amd_circuit_state_count.argtypes = [_VP]
lib.tfhe_amd_circuit_inputs.argtypes = [_VP, ctypes.c_int]
lib.tfhe_amd_circuit_gate.argtypes = [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
lib.tfhe_amd_circuit_lincomb.argtypes = [_VP, ctypes.c_int32, ctypes.c_int32, ctypes.c_int, ctypes.c_int32,
                                         ctypes.c_int, ctypes.c_int32, ctypes.c_int]
lib.tfhe_amd_circuit_info.argtypes = [_VP, _IP, _IP, _IP, _IP]
lib.tfhe_amd_circuit_level_sizes.argtypes = [_VP, _IP, ctypes.c_int]
lib.tfhe_amd_circuit_node.argtypes = [_VP, ctypes.c_int, _IP, _IP, ctypes.POINTER(ctypes.c_int32),
                                      ctypes.POINTER(ctypes.c_int32), _IP]
lib.tfhe_amd_circuit_run_dev.argtypes = [_VP, _VP, ctypes.c_int, _VP, _VP, _VP]
lib.tfhe_amd_circuit_dot.argtypes = [_VP, ctypes.c_int, ctypes.c_int, _IP, _IP, ctypes.c_int, _IP]
lib.tfhe_amd_circuit_compare.argtypes = [_VP, ctypes.c_int, _IP, _IP, ctypes.c_int, ctypes.c_int]
lib.tfhe_amd_circuit_minmax.argtypes = [_VP, ctypes.c_int, _IP, _IP, ctypes.c_int, ctypes.c_int, _IP]
lib.tfhe_amd_circuit_neg.argtypes = [_VP, ctypes.c_int, _IP, _IP]
lib.tfhe_amd_circuit_abs.argtypes = [_VP, ctypes.c_int, _IP, _IP]
lib.tfhe_amd_circuit_divu.argtypes = [_VP, ctypes.c_int, _IP, _IP, _IP, _IP]
lib.tfhe_amd_circuit_div.argtypes = [_VP, ctypes.c_int, _IP, _IP, _IP]
_VPP = ctypes.POINTER(_VP)
lib.tfhe_amd_multi_gate_batch_dev.argtypes = [_VP, ctypes.c_int, _IP] + [_VPP] * 9
lib.tfhe_amd_multi_sync.argtypes = [_VP]
lib.tfhe_amd_multi_circuit_run_dev.argtypes = [_VP, _VP, _IP, _VPP, _VPP, _VPP]
lib.tfhe_amd_multi_circuit_run_host.argtypes = [_VP, _VP, ctypes.c_int, ctypes.c_int, _IP, _I32P, _I32P, ctypes.c_int,
                                                _IP, _I32P, _I32P]
CMP = {"GT": 0, "GE": 1, "LT": 2, "LE": 3, "EQ": 4, "NE": 5}
for _f in ("add", "sub", "add_prefix", "mul"):
    getattr(lib, "tfhe_amd_circuit_" + _f).argtypes = (
        [_VP, ctypes.c_int, _IP, _IP] + ([ctypes.c_int] if _f == "add" else []) + [_IP])


def _ids(v):
    return (ctypes.c_int * len(v))(*[int(x) for x in v])


class Circuit:
    """TfheAmdCircuit: gates over SSA wires, evaluated level by level on the GPU for B
    independent instances (include/tfhe_amd.h, csrc/circuit.cpp)."""

    def __init__(self):
        h = _VP()
        _check(lib.tfhe_amd_circuit_create(ctypes.byref(h)), "circuit_create")
        self.h = h.value

    def close(self):
        if getattr(self, "h", None):
            lib.tfhe_amd_circuit_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def state_count(self):
        """contexts this circuit holds device state for (dropped when a context is destroyed)"""
        return self._w(lib.tfhe_amd_circuit_state_count(self.h), "state_count")

    def _w(self, rc, what):
        if rc < 0:
            raise TfheAmdError(f"{what} failed with code {rc}")
        return rc

    def inputs(self, n):
        first = self._w(lib.tfhe_amd_circuit_inputs(self.h, int(n)), "inputs")
        return list(range(first, first + n))

    def gate(self, name, a, b=-1, c=-1):
        g = GATES[name] if isinstance(name, str) else int(name)
        return self._w(lib.tfhe_amd_circuit_gate(self.h, g, int(a), int(b), int(c)), f"gate {name}")

    def lincomb(self, c0, sa, a, sb=0, b=-1, sc=0, c=-1):
        return self._w(lib.tfhe_amd_circuit_lincomb(self.h, int(c0), int(sa), int(a), int(sb), int(b), int(sc),
                                                    int(c)), "lincomb")

    def _vec(self, fn, a, b, n_out, *extra):
        out = (ctypes.c_int * n_out)()
        rc = getattr(lib, "tfhe_amd_circuit_" + fn)(self.h, len(a), _ids(a), _ids(b), *extra, out)
        self._w(rc, fn)
        return list(out), rc

    def add(self, a, b, carry_in=-1):
        return self._vec("add", a, b, len(a), int(carry_in))

    def sub(self, a, b):
        return self._vec("sub", a, b, len(a))

    def add_prefix(self, a, b):
        return self._vec("add_prefix", a, b, len(a))

    def mul(self, a, b):
        return self._vec("mul", a, b, 2 * len(a))[0]

    def dot(self, a_terms, b_terms, out_bits):
        """sum_t a_t * b_t: a_terms / b_terms are lists of bit-vectors (little-endian wires)"""
        nt, nb = len(a_terms), len(a_terms[0])
        fa = [w for v in a_terms for w in v]
        fb = [w for v in b_terms for w in v]
        out = (ctypes.c_int * out_bits)()
        self._w(lib.tfhe_amd_circuit_dot(self.h, nt, nb, _ids(fa), _ids(fb), int(out_bits), out), "dot")
        return list(out)

    def compare(self, a, b, op, signed=False):
        """one wire: a OP b, OP in GT GE LT LE EQ NE (tfhe_amd_circuit_compare)"""
        return self._w(lib.tfhe_amd_circuit_compare(self.h, len(a), _ids(a), _ids(b), CMP[op], int(signed)),
                       "compare")

    def minmax(self, a, b, want_max=False, signed=False):
        out = (ctypes.c_int * len(a))()
        self._w(lib.tfhe_amd_circuit_minmax(self.h, len(a), _ids(a), _ids(b), int(want_max), int(signed), out),
                "minmax")
        return list(out)

    def neg(self, a):
        out = (ctypes.c_int * len(a))()
        self._w(lib.tfhe_amd_circuit_neg(self.h, len(a), _ids(a), out), "neg")
        return list(out)

    def abs(self, a):
        out = (ctypes.c_int * len(a))()
        self._w(lib.tfhe_amd_circuit_abs(self.h, len(a), _ids(a), out), "abs")
        return list(out)

    def divu(self, a, b):
        q, r = (ctypes.c_int * len(a))(), (ctypes.c_int * len(a))()
        self._w(lib.tfhe_amd_circuit_divu(self.h, len(a), _ids(a), _ids(b), q, r), "divu")
        return list(q), list(r)

    def div(self, a, b):
        q = (ctypes.c_int * len(a))()
        self._w(lib.tfhe_amd_circuit_div(self.h, len(a), _ids(a), _ids(b), q), "div")
        return list(q)

    def info(self):
        v = [ctypes.c_int() for _ in range(4)]
        _check(lib.tfhe_amd_circuit_info(self.h, *[ctypes.byref(x) for x in v]), "circuit_info")
        return dict(zip(("wires", "gates", "bootstraps", "depth"), (x.value for x in v)))

    def level_sizes(self):
        buf = (ctypes.c_int * 4096)()
        n = self._w(lib.tfhe_amd_circuit_level_sizes(self.h, buf, 4096), "level_sizes")
        return list(buf[:n])

    def node(self, w):
        kind, gate = ctypes.c_int(), ctypes.c_int()
        c0 = ctypes.c_int32()
        s = (ctypes.c_int32 * 3)()
        ins = (ctypes.c_int * 3)()
        _check(lib.tfhe_amd_circuit_node(self.h, int(w), ctypes.byref(kind), ctypes.byref(gate), ctypes.byref(c0),
                                         s, ins), "circuit_node")
        return kind.value, gate.value, c0.value, list(s), list(ins)

    def eval_plain(self, bits):
        """Plaintext evaluation of the circuit as built (host; test oracle for the builders):
        wire encodings are +-2^29 and every bootstrapped row is the sign of its torus sum,
        so the threshold gates are checked in the same arithmetic the GPU rows use.
        bits: {input wire: 0/1 array}; returns {wire: 0/1 array} for all wires."""
        e8 = 1 << 29
        n_w = self.info()["wires"]
        val = {}

        def enc(w):
            return val[w]
        spec = {0: (e8, -1, -1), 1: (e8, 1, 1), 2: (-e8, 1, 1), 3: (1 << 30, 2, 2), 4: (-(1 << 30), -2, -2),
                5: (-e8, -1, -1), 6: (-e8, -1, 1), 7: (-e8, 1, -1), 8: (e8, -1, 1), 9: (e8, 1, -1)}

        def sign(x):   # torus phase > 0 (int32)
            x = (np.asarray(x, dtype=np.int64) + 2**31) % 2**32 - 2**31
            return np.where(x > 0, e8, -e8).astype(np.int64)
        for w in range(n_w):
            kind, gate, c0, s, ins = self.node(w)
            if kind == 0:
                val[w] = np.where(np.asarray(bits[w]) != 0, e8, -e8).astype(np.int64)
            elif kind == 2:
                if gate == GATES["CONST"]:
                    val[w] = np.int64(c0)
                else:
                    val[w] = (-1 if gate == GATES["NOT"] else 1) * enc(ins[0])
            elif gate == GATES["MUX"]:
                u1 = sign(-e8 + enc(ins[0]) + enc(ins[1]))
                u2 = sign(-e8 - enc(ins[0]) + enc(ins[2]))
                val[w] = sign(e8 + u1 + u2)
            else:
                if gate in spec:
                    c, sa, sb = spec[gate]
                    x = c + sa * enc(ins[0]) + sb * enc(ins[1])
                else:
                    x = c0 + sum(s[t] * enc(ins[t]) for t in range(3) if ins[t] >= 0)
                val[w] = sign(x)
        return {w: (np.asarray(v) > 0).astype(np.int64) for w, v in val.items()}

    def run(self, ctx, B, inputs, outputs, keyset, rng, stream=None):
        """Encrypt `inputs` ({wire: bit array [B]}), run on the GPU, decrypt `outputs`
        (list of wires) -> {wire: bit array}.  Convenience for tests and the bench."""
        import torch
        n_w = self.info()["wires"]
        wa = torch.zeros((n_w, B, n_lwe), dtype=torch.int32, device="cuda")
        wb = torch.zeros((n_w, B), dtype=torch.int32, device="cuda")
        for w, bits in inputs.items():
            a, b = keyset.encrypt(np.asarray(bits), rng)
            wa[w] = torch.from_numpy(a).cuda()
            wb[w] = torch.from_numpy(b).cuda()
        self.run_dev(ctx, B, wa, wb, stream)
        torch.cuda.synchronize()
        ha, hb = wa.cpu().numpy(), wb.cpu().numpy()
        return {w: keyset.decrypt(ha[w], hb[w]) for w in outputs}

    def run_dev(self, ctx, B, wa, wb, stream=None):
        _check(lib.tfhe_amd_circuit_run_dev(ctx.h, self.h, int(B), wa.data_ptr(), wb.data_ptr(), stream),
               "circuit_run_dev")


def bits_of(x, nbits):
    """little-endian bit planes of an integer array: [nbits][B]"""
    x = np.asarray(x, dtype=np.int64)
    return [((x >> i) & 1) for i in range(nbits)]


def int_of(planes):
    return sum(np.asarray(p, dtype=np.int64) << i for i, p in enumerate(planes))
