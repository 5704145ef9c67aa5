"""Tier-1 TFHE C API from many threads and in place: the reference's callers
enter the gates from OpenMP threads and pass results that alias inputs.  The driver
(tests/callers/tier1_threads.cpp) is built by __graft_entry__.build() through
tests/callers/Makefile against include/ + libtfhe_amd alone."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CALLERS = os.path.join(REPO, "tests", "callers")
EXE = os.path.join(CALLERS, "_bin", "tier1_threads")
LIB = os.path.join(REPO, "cpu-gpu-tfhe_amd", "lib", "libtfhe_amd.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="libtfhe_amd.so not built")
def test_tier1_driver_builds():
    """The driver compiles and links against the public headers and the library alone."""
    subprocess.check_call(["make", "-s", "-C", CALLERS])
    assert os.access(EXE, os.X_OK)


@pytest.mark.gpu
@pytest.mark.parametrize("keyrows", ["uniform", "nonuniform"])
def test_tier1_threads_and_aliasing_gpu(keyrows):
    """Every gate + MUX: sequential vs 8 OpenMP threads vs result aliasing an input vs 8 threads with
    the kinds interleaved (the queue's batches mix kinds, MUX included) give the same samples word
    for word and current_variance bit for bit (the mixed batches' device-side variance sum against
    the same gate run alone), on a key with the reference's equal key-switching-key row
    variances and on one whose rows differ; every output decrypts to its truth table; 16 short-lived
    threads running one gate each leave the key's lane count unchanged."""
    assert os.access(EXE, os.X_OK), "tests/callers/_bin/tier1_threads missing: run __graft_entry__.build()"
    r = subprocess.run([EXE, "24"] + (["nonuniform"] if keyrows == "nonuniform" else []),
                       capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, (r.returncode, r.stderr[-2000:])
    out = json.loads(lines[-1])
    assert r.returncode == 0, (out, r.stderr[-2000:])
    assert out["par_mismatch"] == 0 and out["alias_mismatch"] == 0 and out["truth_errors"] == 0, out
    assert out["mixed_mismatch"] == 0 and out["zero_variance"] == 0, out
    assert out["nonuniform_key"] == (keyrows == "nonuniform"), out
    # threads that exit give their lanes back (no stream / scratch / pinned-memory leak per thread)
    assert out["short_thread_errors"] == 0 and out["lanes_after_short_threads"] == out["lanes_before"], out


def _rate_run(env_extra, args):
    exe = os.path.join(CALLERS, "_bin", "tier1_rate")
    assert os.access(exe, os.X_OK), "tests/callers/_bin/tier1_rate missing: run __graft_entry__.build()"
    env = dict(os.environ, **env_extra)
    r = subprocess.run([exe] + [str(a) for a in args], capture_output=True, text=True, timeout=300, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, (r.returncode, r.stderr[-2000:])
    out = json.loads(lines[-1])
    assert r.returncode == 0, (out, r.stderr[-2000:])
    return out


@pytest.mark.gpu
def test_tier1_coalescing_queue_rate():
    """Concurrent single-gate calls (OpenMP teams of 1, 8 and 64 threads, half of them in place)
    through the coalescing queue: every output equals the sequential result word for word, and 64
    threads reach >= 20x the one-thread gate rate; the per-thread-lane path
    (TFHE_AMD_TIER1_COALESCE=0) is measured beside it."""
    q = _rate_run({}, [16, 1, 8, 64])
    lanes = _rate_run({"TFHE_AMD_TIER1_COALESCE": "0"}, [16, 1, 8, 64])
    print(json.dumps({"queue": q, "per_thread_lanes": lanes}))
    for out in (q, lanes):
        assert out["truth_errors"] == 0 and out["mismatches"] == 0, out
    rate = {r["threads"]: r["gates_per_s"] for r in q["runs"]}
    assert rate[64] >= 20 * rate[1], q
    # mixed gate kinds (all 10 binary gates and MUX across the team): one launch per batch
    assert q["mixed_kinds"]["mismatches"] == 0 and q["mixed_kinds"]["gates_per_s"] >= 10 * rate[1], q
    assert max(r["largest_batch"] for r in q["runs"]) > 1, q


@pytest.mark.gpu
def test_tier1_single_gate_latency():
    """Sequential single-gate calls through the C API (what an unchanged Cipher.cpp caller sees):
    chained bootsNAND decrypt right and cost about one B = 1 device step (1.7 ms) plus the
    synchronous host round trip and the current_variance bookkeeping."""
    exe = os.path.join(CALLERS, "_bin", "tier1_latency")
    assert os.access(exe, os.X_OK), "tests/callers/_bin/tier1_latency missing: run __graft_entry__.build()"
    r = subprocess.run([exe, "20"], capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines and r.returncode == 0, (r.returncode, r.stdout[-500:], r.stderr[-2000:])
    out = json.loads(lines[-1])
    print(out)
    assert out["decrypt_ok"] and out["tier1_ms_per_gate"] < 5.0, out


@pytest.mark.gpu
def test_tier1_current_variance_as_reference(keyset, okey, rng):
    """current_variance after bootsNAND / bootsMUX (Tier-1, through the C ABI): the reference's
    lweKeySwitch restarts it at 0 and adds the variance of every key-switching-key row its
    non-zero digits select (lwe-keyswitch-functions.cu:101-127, 955-987; lwe-functions.cu:150),
    in i, j order — recomputed here from the oracle's exact key-switch input and the row
    variances of the key's own structs."""
    import ctypes
    import numpy as np
    import tfhe_amd as T

    class LweSample(ctypes.Structure):
        _fields_ = [("a", ctypes.POINTER(ctypes.c_int32)), ("b", ctypes.c_int32), ("current_variance", ctypes.c_double)]
    P = ctypes.c_void_p
    lib = T.lib
    lib.bootsNAND.argtypes = [P, P, P, P]
    lib.bootsMUX.argtypes = [P, P, P, P, P]
    cloud = keyset.cloud
    bkfft = P.from_address(cloud + 16).value                 # cloud->bkFFT
    ks = P.from_address(bkfft + 40).value                    # bkFFT->ks
    ks0 = P.from_address(ks + 24).value                      # ks->ks0_raw
    rows = (LweSample * (1024 * 8 * 4)).from_address(ks0)
    row_var = np.array([rows[r].current_variance for r in range(1024 * 8 * 4)])

    def expected(u_a):
        v = 0.0
        for i in range(1024):
            aibar = (int(u_a[i]) + (1 << 15)) & 0xFFFFFFFF
            for j in range(8):
                aij = (aibar >> (30 - 2 * j)) & 3
                if aij:
                    v += row_var[(i * 8 + j) * 4 + aij]
        return v

    arr = lib.new_gate_bootstrapping_ciphertext_array(4, P(keyset.params))
    s = (LweSample * 4).from_address(arr)
    bits = rng.integers(0, 2, 3)
    enc = [keyset.encrypt(np.array([x]), rng) for x in bits]
    for k, (a, b) in enumerate(enc):
        ctypes.memmove(s[k].a, a[0].ctypes.data, 4 * 500)
        s[k].b = int(b[0])
    addr = [ctypes.addressof(s[k]) for k in range(4)]
    lib.bootsNAND(P(addr[3]), P(addr[0]), P(addr[1]), P(cloud))
    t_a = (-(enc[0][0][0].astype(np.int64)) - enc[1][0][0]).astype(np.int64)
    t_b = np.int64(1 << 29) - enc[0][1][0] - enc[1][1][0]
    u_a, _ = okey.woks_batch(1 << 29, t_a[None, :], np.array([t_b]))
    assert s[3].current_variance == expected(u_a[0]) and s[3].current_variance > 0
    lib.bootsMUX(P(addr[3]), P(addr[0]), P(addr[1]), P(addr[2]), P(cloud))
    u1, _ = okey.woks_batch(1 << 29, (enc[0][0][0].astype(np.int64) + enc[1][0][0])[None, :],
                            np.array([np.int64(-(1 << 29)) + enc[0][1][0] + enc[1][1][0]]))
    u2, _ = okey.woks_batch(1 << 29, (-enc[0][0][0].astype(np.int64) + enc[2][0][0])[None, :],
                            np.array([np.int64(-(1 << 29)) - enc[0][1][0] + enc[2][1][0]]))
    usum = (u1[0].astype(np.int64) + u2[0]).astype(np.int64)
    assert s[3].current_variance == expected(usum)
    lib.delete_gate_bootstrapping_ciphertext_array(4, arr)


@pytest.mark.gpu
def test_current_variance_nonuniform_key_rows(rng):
    """The device-side current_variance sum has two forms (keyswitch.hip k_ks_variance): a table of
    the sequential sums of k equal terms when every key-switching-key row carries the same variance
    (the reference's lweCreateKeySwitchKey), and the full sequential sum otherwise.  A key whose row
    variances are made unequal before its first gate takes the second form; bootsNAND (Tier-1 queue)
    and tfhe_amd_boots_batch (record path, 3 gates) must still give the reference's double exactly."""
    import ctypes
    import numpy as np
    import oracle_ctypes as O
    import tfhe_amd as T

    class LweSample(ctypes.Structure):
        _fields_ = [("a", ctypes.POINTER(ctypes.c_int32)), ("b", ctypes.c_int32), ("current_variance", ctypes.c_double)]
    P = ctypes.c_void_p
    lib = T.lib
    lib.bootsNAND.argtypes = [P, P, P, P]
    lib.tfhe_amd_boots_batch.argtypes = [ctypes.c_int, P, P, P, P, ctypes.c_int, P]
    K = T.SecretKeyset(seed=(27, 18, 28))
    ok = O.OracleKey(K.bk, K.ksk, use_ntt=True)
    try:
        cloud = K.cloud
        bkfft = P.from_address(cloud + 16).value
        ks = P.from_address(bkfft + 40).value
        rows = (LweSample * (1024 * 8 * 4)).from_address(P.from_address(ks + 24).value)
        for r in range(1024 * 8 * 4):   # unequal rows, before the key's device tables exist
            rows[r].current_variance *= 1.0 + ((r * 37) % 11) * 1e-3
        row_var = np.array([rows[r].current_variance for r in range(1024 * 8 * 4)])

        def expected(u):
            v = 0.0
            for i in range(1024):
                aibar = (int(u[i]) + (1 << 15)) & 0xFFFFFFFF
                for j in range(8):
                    aij = (aibar >> (30 - 2 * j)) & 3
                    if aij:
                        v += row_var[(i * 8 + j) * 4 + aij]
            return v

        B = 3
        arrs = [lib.new_gate_bootstrapping_ciphertext_array(B, P(K.params)) for _ in range(3)]
        s = [(LweSample * B).from_address(p) for p in arrs]
        enc = [K.encrypt(rng.integers(0, 2, B), rng) for _ in range(2)]
        for k in range(2):
            for i in range(B):
                ctypes.memmove(s[k][i].a, enc[k][0][i].ctypes.data, 4 * 500)
                s[k][i].b = int(enc[k][1][i])
        t_a = (-(enc[0][0].astype(np.int64)) - enc[1][0]).astype(np.int64)
        t_b = np.int64(1 << 29) - enc[0][1].astype(np.int64) - enc[1][1]
        u_a, _ = ok.woks_batch(1 << 29, t_a, t_b)
        lib.bootsNAND(P(ctypes.addressof(s[2][0])), P(ctypes.addressof(s[0][0])), P(ctypes.addressof(s[1][0])), P(cloud))
        assert s[2][0].current_variance == expected(u_a[0]) > 0
        assert lib.tfhe_amd_boots_batch(T.GATES["NAND"], P(arrs[2]), P(arrs[0]), P(arrs[1]), None, B, P(cloud)) == 0
        for i in range(B):
            assert s[2][i].current_variance == expected(u_a[i]), i
        for p in arrs:
            lib.delete_gate_bootstrapping_ciphertext_array(B, P(p))
    finally:
        del ok
        K.close()


@pytest.mark.gpu
def test_boots_batch_lwesample_arrays(keyset, ctx, rng):
    """tfhe_amd_boots_batch over LweSample arrays (SURVEY.md §8(b)'s LweSample convenience overload):
    1 100 NAND gates (two pipelined slices: 1 024 + 76) and 33 MUX gates give the Torus32 words of
    the device batch path, also in place (result = the first input array), and current_variance —
    summed on the device by k_ks_variance in the reference's order of double adds — equals, bit for
    bit, the single Tier-1 gates' on sampled rows (test_tier1_current_variance_as_reference pins
    those to the reference's sum)."""
    import ctypes
    import time
    import numpy as np
    import tfhe_amd as T

    class LweSample(ctypes.Structure):
        _fields_ = [("a", ctypes.POINTER(ctypes.c_int32)), ("b", ctypes.c_int32), ("current_variance", ctypes.c_double)]
    P = ctypes.c_void_p
    lib = T.lib
    lib.tfhe_amd_boots_batch.argtypes = [ctypes.c_int, P, P, P, P, ctypes.c_int, P]
    lib.bootsNAND.argtypes = [P, P, P, P]
    lib.bootsMUX.argtypes = [P, P, P, P, P]
    lib.new_gate_bootstrapping_ciphertext_array.restype = P
    cloud = keyset.cloud

    def arrays(B, n):
        out = []
        for _ in range(n):
            p = lib.new_gate_bootstrapping_ciphertext_array(B, P(keyset.params))
            out.append((p, (LweSample * B).from_address(p)))
        return out

    def fill(s, a, b):
        for k in range(a.shape[0]):
            ctypes.memmove(s[k].a, a[k].ctypes.data, 4 * 500)
            s[k].b = int(b[k])

    for gate, B in (("NAND", 1100), ("MUX", 33)):
        nin = 3 if gate == "MUX" else 2
        bits = [rng.integers(0, 2, B) for _ in range(nin)]
        host = [keyset.encrypt(v, rng) for v in bits]
        arrs = arrays(B, nin + 1)
        for (p, s), (a, b) in zip(arrs[:nin], host):
            fill(s, a, b)
        res_p, res = arrs[nin]
        dts = []
        for _ in range(3):   # the first call also sizes the context's staging and variance buffers
            t0 = time.perf_counter()
            rc = lib.tfhe_amd_boots_batch(T.GATES[gate], P(res_p), P(arrs[0][0]), P(arrs[1][0]),
                                          P(arrs[2][0]) if nin == 3 else None, B, P(cloud))
            dts.append(time.perf_counter() - t0)
            assert rc == 0
        got_a = np.array([np.ctypeslib.as_array(res[k].a, (500,)) for k in range(B)])
        got_b = np.array([res[k].b for k in range(B)], dtype=np.int32)
        want = ctx.gate_host(gate, *[v for hb in host for v in hb])
        assert np.array_equal(got_a, want[0]) and np.array_equal(got_b, want[1]), gate
        print(f"tfhe_amd_boots_batch {gate} B={B}: {min(dts[1:]) * 1e3:.2f} ms warm ({dts[0] * 1e3:.1f} ms first)")
        one = arrays(1, 1)[0]
        for k in np.unique(np.concatenate([[0, B - 1, min(1023, B - 1), min(1024, B - 1)],
                                           rng.choice(B, 12, replace=False)])):
            ins = [P(ctypes.addressof(arrs[j][1][k])) for j in range(nin)]
            (lib.bootsMUX if gate == "MUX" else lib.bootsNAND)(P(one[0]), *ins, P(cloud))
            assert one[1][0].current_variance == res[k].current_variance > 0, (gate, k)
        # in place: the result array is the first input array (slices of 1 024 + 76 alias row by row)
        rc = lib.tfhe_amd_boots_batch(T.GATES[gate], P(arrs[0][0]), P(arrs[0][0]), P(arrs[1][0]),
                                      P(arrs[2][0]) if nin == 3 else None, B, P(cloud))
        assert rc == 0
        got_a = np.array([np.ctypeslib.as_array(arrs[0][1][k].a, (500,)) for k in range(B)])
        got_b = np.array([arrs[0][1][k].b for k in range(B)], dtype=np.int32)
        assert np.array_equal(got_a, want[0]) and np.array_equal(got_b, want[1]), (gate, "in place")
        assert all(arrs[0][1][k].current_variance == res[k].current_variance for k in range(B))
        for p, _ in arrs + [one]:
            lib.delete_gate_bootstrapping_ciphertext_array(B if p != one[0] else 1, P(p))


@pytest.mark.gpu
def test_tier1_raw_bootstrap_exports(keyset, okey, rng):
    """The raw Tier-1 exports Cipher.cpp calls directly (addBitsRaw / bootsANDXOR, Cipher.cpp:647-766;
    SURVEY.md §8(b)): tfhe_bootstrap_woKS_FFT (dimension-1 024 output), tfhe_bootstrap_FFT and
    lweKeySwitch, through the C ABI on the key's own LweBootstrappingKeyFFT / LweKeySwitchKey
    structs, against the exact oracle word for word — several mu (the gates' 1/8 and others), an
    all-zero mask (identity CMux steps), modswitch edges, and tfhe_bootstrap_FFT with the result
    aliasing its input."""
    import ctypes
    import numpy as np
    import tfhe_amd as T

    class LweSample(ctypes.Structure):
        _fields_ = [("a", ctypes.POINTER(ctypes.c_int32)), ("b", ctypes.c_int32), ("current_variance", ctypes.c_double)]
    P = ctypes.c_void_p
    lib = T.lib
    lib.tfhe_bootstrap_woKS_FFT.argtypes = [P, P, ctypes.c_int32, P]
    lib.tfhe_bootstrap_FFT.argtypes = [P, P, ctypes.c_int32, P]
    lib.lweKeySwitch.argtypes = [P, P, P]
    bkfft = P.from_address(keyset.cloud + 16).value          # cloud->bkFFT
    ks = P.from_address(bkfft + 40).value                    # bkFFT->ks

    def sample(n, a=None, b=0):
        buf = np.zeros(n, np.int32) if a is None else np.ascontiguousarray(a, dtype=np.int32).copy()
        s = LweSample()
        s.a = buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        s.b = int(b)
        return s, buf

    bits = rng.integers(0, 2, 6)
    x_a, x_b = keyset.encrypt(bits, rng)
    x_a = x_a.copy()
    x_a[3, :] = 0                                    # every rotation amount 0 (identity CMux steps)
    x_a[4, :4] = [1 << 21, -(1 << 21), 2**31 - 1, -(2**31)]   # modswitch edges
    mus = [1 << 29, -(1 << 29), 1 << 30, 123456789]
    for k in range(x_a.shape[0]):
        mu = mus[k % len(mus)]
        xs, _ = sample(500, x_a[k], x_b[k])
        # woKS: the extracted dimension-1 024 sample
        u, ubuf = sample(1024)
        lib.tfhe_bootstrap_woKS_FFT(P(ctypes.addressof(u)), P(bkfft), mu, P(ctypes.addressof(xs)))
        w_a, w_b = okey.woks_batch(mu, x_a[k:k + 1], x_b[k:k + 1])
        assert np.array_equal(ubuf, w_a[0]) and u.b == int(w_b[0]), ("woKS", k)
        # full bootstrap = woKS + key switch
        r, rbuf = sample(500)
        lib.tfhe_bootstrap_FFT(P(ctypes.addressof(r)), P(bkfft), mu, P(ctypes.addressof(xs)))
        k_a, k_b = okey.keyswitch_batch(w_a, w_b)
        assert np.array_equal(rbuf, k_a[0]) and r.b == int(k_b[0]), ("bootstrap", k)
        # the standalone key switch on the woKS output
        r2, r2buf = sample(500)
        lib.lweKeySwitch(P(ctypes.addressof(r2)), P(ks), P(ctypes.addressof(u)))
        assert np.array_equal(r2buf, k_a[0]) and r2.b == int(k_b[0]), ("lweKeySwitch", k)
        # result aliasing the input sample
        xa, xabuf = sample(500, x_a[k], x_b[k])
        lib.tfhe_bootstrap_FFT(P(ctypes.addressof(xa)), P(bkfft), mu, P(ctypes.addressof(xa)))
        assert np.array_equal(xabuf, k_a[0]) and xa.b == int(k_b[0]), ("aliased bootstrap", k)
