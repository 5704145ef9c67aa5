"""Key / ciphertext files (include/tfhe/tfhe_io.h) — SURVEY.md §8(f) row 2.

The reference's writer (gpuParallel/tfhe_io.cu) needs cufftXt.h and cannot be built here,
so the byte format is pinned by an independent numpy restatement of tfhe_io.cu /
tfhe_generic_streams.cu below (`parse_*`), applied to what libtfhe_amd writes, plus
round trips and the reference's own callers (cpuParallel/main.cpp, cloud.cpp, Cipher.cpp)
compiled unchanged against include/ (oracle/build_callers.sh).
"""
import json
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

import tfhe_amd as T

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CALLERS = os.path.join(REPO, "oracle", "_ref", "callers")
REF_CALLERS = "/root/reference/cpuParallel"

KS_STDEV = 2.4349504419032758e-05
BK_STDEV = 7.180961047225788e-09
MAX_STDEV = 0.012466946262544772

# ---------------------------------------------------------------- format restatement

PARAM_SECTIONS = [   # (title, sorted "name: value" lines), tfhe_io.cu:1014-1035, std::map order
    ("GATEBOOTSPARAMS", [("ks_basebit", "2"), ("ks_t", "8")]),
    ("LWEPARAMS", [("alpha_max", "%.8f" % MAX_STDEV), ("alpha_min", "%.8f" % KS_STDEV), ("n", "500")]),
    ("TLWEPARAMS", [("N", "1024"), ("alpha_max", "%.8f" % MAX_STDEV), ("alpha_min", "%.8f" % BK_STDEV), ("k", "1")]),
    ("TGSWPARAMS", [("Bgbit", "10"), ("l", "2")]),
]
KS_SECTION = ("LWEKSPARAMS", [("basebit", "2"), ("n", "1024"), ("t", "8")])


def section_text(title, kv):
    return ("-----BEGIN %s-----\n" % title + "".join("%s: %s\n" % e for e in kv) +
            "-----END %s-----\n" % title).encode()


class Reader:
    def __init__(self, buf):
        self.buf, self.pos = buf, 0

    def section(self):
        """new_TextModeProperties_fromIstream (tfhe_generic_streams.cu:136-170)."""
        title, kv = None, {}
        while True:
            end = self.buf.index(b"\n", self.pos)
            line = self.buf[self.pos:end].decode()
            self.pos = end + 1
            if line.startswith("-----BEGIN ") and line.endswith("-----"):
                title = line[11:-5]
            elif title is not None and line == "-----END %s-----" % title:
                return title, kv
            elif title is not None and ": " in line:
                k, v = line.split(": ", 1)
                kv[k] = v

    def take(self, dtype, count=1):
        a = np.frombuffer(self.buf, dtype=dtype, count=count, offset=self.pos)
        self.pos += a.nbytes
        return a if count != 1 else a[0]


def parse_keyfile(buf, secret):
    """cloud key: params, LWEKSPARAMS, KSK content (uid 200), BK content (uid 201)
    (tfhe_io.cu:757-788, 883-909, 937-945, 1099-1103); secret adds lwe key (uid 43) and
    tgsw key (uid 169) (:1160-1166)."""
    r = Reader(buf)
    secs = [r.section() for _ in range(5)]
    out = {"sections": secs}
    assert r.take("<i4") == 200
    out["ksk_var"] = r.take("<f8")
    out["ksk"] = r.take("<i4", 1024 * 8 * 4 * 501).reshape(1024, 8, 4, 501)
    assert r.take("<i4") == 201
    out["bk_var"] = r.take("<f8")
    out["bk"] = r.take("<i4", 500 * 4 * 2 * 1024).reshape(500, 4, 2, 1024)
    if secret:
        assert r.take("<i4") == 43
        out["lwe_key"] = r.take("<i4", 500)
        assert r.take("<i4") == 169
        out["tlwe_key"] = r.take("<i4", 1024)
    assert r.pos == len(buf)
    return out


def ciphertext_bytes(a, b, var):
    """write_lweSample (tfhe_io.cu:101-108): i32 42, a[n], b, f64 variance."""
    out = b""
    for i in range(a.shape[0]):
        out += np.int32(42).tobytes() + a[i].astype("<i4").tobytes() + np.int32(b[i]).astype("<i4").tobytes() \
            + np.float64(var[i]).astype("<f8").tobytes()
    return out


# ---------------------------------------------------------------- tests

@pytest.fixture(scope="module")
def files(keyset, tmp_path_factory):
    d = tmp_path_factory.mktemp("keys")
    keyset.save(str(d / "secret.key"))
    keyset.save_cloud(str(d / "cloud.key"))
    return d


def test_header_text_exact(files):
    buf = open(files / "cloud.key", "rb").read()
    want = b"".join(section_text(t, kv) for t, kv in PARAM_SECTIONS + [KS_SECTION])
    assert buf[:len(want)] == want


@pytest.mark.parametrize("secret", [False, True])
def test_keyfile_layout(files, keyset, secret):
    buf = open(files / ("secret.key" if secret else "cloud.key"), "rb").read()
    p = parse_keyfile(buf, secret)
    assert [s[0] for s in p["sections"]] == [t for t, _ in PARAM_SECTIONS] + ["LWEKSPARAMS"]
    np.testing.assert_array_equal(p["ksk"], keyset.ksk)
    np.testing.assert_array_equal(p["bk"], keyset.bk)
    # max variance over samples: KSK rows alpha^2 (h = 0 rows are noiseless), BK rows alpha^2
    assert p["ksk_var"] == KS_STDEV ** 2
    assert p["bk_var"] == BK_STDEV ** 2
    if secret:
        np.testing.assert_array_equal(p["lwe_key"], keyset.lwe_key)
        np.testing.assert_array_equal(p["tlwe_key"], keyset.tlwe_key)


def test_secret_roundtrip_bytes(files, tmp_path):
    K2 = T.SecretKeyset(path=str(files / "secret.key"))
    try:
        K2.save(str(tmp_path / "again.key"))
        K2.save_cloud(str(tmp_path / "again_cloud.key"))
    finally:
        K2.close()
    assert open(tmp_path / "again.key", "rb").read() == open(files / "secret.key", "rb").read()
    assert open(tmp_path / "again_cloud.key", "rb").read() == open(files / "cloud.key", "rb").read()


def test_cloud_roundtrip(files, keyset, tmp_path):
    C = T.CloudKeyset(str(files / "cloud.key"))
    try:
        np.testing.assert_array_equal(C.export_bk(), keyset.bk)
        np.testing.assert_array_equal(C.export_ksk(), keyset.ksk)
        C.save(str(tmp_path / "c2.key"))
    finally:
        C.close()
    assert open(tmp_path / "c2.key", "rb").read() == open(files / "cloud.key", "rb").read()


def test_ciphertexts(keyset, rng, tmp_path):
    bits = rng.integers(0, 2, 20)
    a, b = keyset.encrypt(bits, rng)
    var = np.full(20, KS_STDEV ** 2)
    path = str(tmp_path / "cloud.data")
    T.write_ciphertexts(path, keyset.params, a, b, variance=KS_STDEV ** 2)
    assert open(path, "rb").read() == ciphertext_bytes(a, b, var)
    a2, b2, v2 = T.read_ciphertexts(path, keyset.params, 20)
    np.testing.assert_array_equal(a2, a)
    np.testing.assert_array_equal(b2, b)
    np.testing.assert_array_equal(v2, var)
    np.testing.assert_array_equal(keyset.decrypt(a2, b2), bits)


_ABORT_SNIPPET = r"""
import ctypes, sys
L = ctypes.CDLL(sys.argv[1]); libc = ctypes.CDLL(None)
libc.fopen.restype = ctypes.c_void_p; libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
fn = getattr(L, sys.argv[3]); fn.restype = ctypes.c_void_p; fn.argtypes = [ctypes.c_void_p]
print("ptr", fn(libc.fopen(sys.argv[2].encode(), b"rb")))
"""


def _load_in_child(path, fn):
    return subprocess.run([sys.executable, "-c", _ABORT_SNIPPET, T.LIB_PATH, str(path), fn],
                          capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("corrupt", ["uid", "title", "shape", "truncated"])
def test_bad_files_abort(files, tmp_path, corrupt):
    """Wrong uid / wrong section / non-default shape / short file: abort like the reference
    (abort() / die_dramatically, tfhe_io.cu:805-806, 925-926, 1025)."""
    buf = bytearray(open(files / "cloud.key", "rb").read())
    hdr = b"".join(section_text(t, kv) for t, kv in PARAM_SECTIONS + [KS_SECTION])
    if corrupt == "uid":
        buf[len(hdr):len(hdr) + 4] = np.int32(201).tobytes()
    elif corrupt == "title":
        buf = bytearray(bytes(buf).replace(b"TGSWPARAMS", b"TLWEPARAMS", 2))
    elif corrupt == "shape":
        buf = bytearray(bytes(buf).replace(b"n: 500\n", b"n: 630\n", 1))
    else:
        buf = buf[:len(buf) - 4096]
    p = tmp_path / "bad.key"
    p.write_bytes(bytes(buf))
    r = _load_in_child(p, "new_tfheGateBootstrappingCloudKeySet_fromFile")
    assert r.returncode != 0 and "ptr" not in r.stdout, (r.returncode, r.stdout, r.stderr[-400:])


def test_good_file_loads_in_child(files):
    r = _load_in_child(files / "cloud.key", "new_tfheGateBootstrappingCloudKeySet_fromFile")
    assert r.returncode == 0 and "ptr" in r.stdout, r.stderr[-400:]


# ---------------------------------------------------------------- the reference's callers

def _callers_built():
    return all(os.path.exists(os.path.join(CALLERS, b)) for b in ("main", "cloud", "cipher_ops"))


@pytest.mark.skipif(not os.path.isdir(REF_CALLERS), reason="reference sources not present")
def test_reference_callers_compile_unchanged():
    """cpuParallel/main.cpp, cloud.cpp and Cipher.cpp build against include/ + libtfhe_amd
    with only the include/link lines of compile.sh changed."""
    subprocess.check_call(["bash", os.path.join(REPO, "oracle", "build_callers.sh")])
    assert _callers_built()


@pytest.mark.skipif(not os.path.isdir(REF_CALLERS), reason="reference sources not present")
def test_reference_main_writes_readable_files(tmp_path):
    """Run the reference's client (main.cpp: keygen seed {314,1592,657}, encrypt 10 and 2,
    export secret.key / cloud.key / cloud.data); read everything back through our loader."""
    if not _callers_built():
        subprocess.check_call(["bash", os.path.join(REPO, "oracle", "build_callers.sh")])
    subprocess.run([os.path.join(CALLERS, "main"), "10", "2"], cwd=tmp_path, check=True, timeout=300,
                   capture_output=True)
    K = T.SecretKeyset(path=str(tmp_path / "secret.key"))
    try:
        a, b, _ = T.read_ciphertexts(str(tmp_path / "cloud.data"), K.params, 32)
        bits = K.decrypt(a, b)
        assert sum(int(bits[i]) << i for i in range(16)) == 10
        assert sum(int(bits[16 + i]) << i for i in range(16)) == 2
        ref = T.SecretKeyset()          # same seed, same RNG stream -> same keys
        try:
            np.testing.assert_array_equal(K.bk, ref.bk)
            np.testing.assert_array_equal(K.lwe_key, ref.lwe_key)
        finally:
            ref.close()
    finally:
        K.close()


@pytest.mark.gpu
def test_reference_callers_gpu(tmp_path):
    """The reference's Cipher circuits (ripple-carry add, two's-complement subtract,
    shift-and-add multiply, minimum, ==, >) run on the MI355X engine through the unchanged
    TFHE API, on keys and ciphertexts from the reference's main.cpp."""
    if not _callers_built():
        pytest.skip("oracle/_ref/callers not built (needs the reference sources at build time)")
    subprocess.run([os.path.join(CALLERS, "main"), "1234", "567"], cwd=tmp_path, check=True, timeout=300,
                   capture_output=True)
    r = subprocess.run([os.path.join(CALLERS, "cipher_ops")], cwd=tmp_path, capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    a, b = 1234, 567
    assert out["a"] == a and out["b"] == b
    assert out["sum"] == a + b
    assert out["diff"] == a - b
    assert out["prod"] == (a & 0xFF) * (b & 0xFF)
    assert out["min"] == min(a, b)
    assert out["eq"] == 0 and out["gt"] == 1


def test_host_api_surface_streams_and_helpers():
    """The host-side TFHE API a libtfhe user may call beyond the reference's callers
    (tests/callers/api_misc.cpp, built by __graft_entry__.build() against include/ + the library):
    the std::stream writers give the FILE* writers' bytes and read back to identical keys / samples
    (parameter set, secret and cloud keysets, gate ciphertexts, single LweSamples), the
    allocators, lweClear, lweSymEncryptWithExternalNoise (phase = message + dtot32(noise), as
    lwe-functions.cu:53-64) and t32tod."""
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "callers", "_bin", "api_misc")
    if not os.access(exe, os.X_OK):
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(os.path.dirname(exe))])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, (r.returncode, r.stderr[-2000:])
    out = json.loads(lines[-1])
    assert r.returncode == 0 and out["failed"] == 0, out
