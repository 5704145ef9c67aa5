"""Several devices on the MI355X: the library's multi-device context
(tfhe_amd_multi_*: one key replica and worker thread per device, contiguous shards) and the
SURVEY §8(b) Tier-2 names tfhe_gpu_init / tfhe_gpu_boots_batch, through the C ABI.  A single-GPU
box exercises the split with several contexts on device 0 (the device list may repeat a device);
with more GPUs visible the same batch also runs over all of them.  The per-process path
(torchrun, one rank per GPU) is rehearsed with two ranks evaluating their shards on cuda:0."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle_ctypes as O
import tfhe_amd as T

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


def test_multi_context_split_bit_exact(ctx, okey, keyset, rng):
    """Three contexts on device 0: a ragged batch of 301 gates (101 + 100 + 100) and a MUX
    batch come back word for word as from one context, and match the oracle on the seams."""
    m = T.MultiContext(keyset.bk, keyset.ksk, [0, 0, 0])
    try:
        B = 301
        x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
        host = keyset.encrypt(x, rng) + keyset.encrypt(y, rng)
        got = m.gate_host("XOR", *host)
        one = ctx.gate_host("XOR", *host)
        assert np.array_equal(got[0], one[0]) and np.array_equal(got[1], one[1])
        assert np.array_equal(keyset.decrypt(*got), x ^ y)
        idx = np.array([0, 100, 101, 200, 201, 300])
        o = okey.gate_batch("XOR", *(v[idx] for v in host))
        assert np.array_equal(got[0][idx], o[0]) and np.array_equal(got[1][idx], o[1])
        s, u, v = (rng.integers(0, 2, 40) for _ in range(3))
        (sa, sb), (ua, ub), (va, vb) = (keyset.encrypt(w, rng) for w in (s, u, v))
        mux = m.gate_host("MUX", sa, sb, ua, ub, va, vb)
        assert np.array_equal(keyset.decrypt(*mux), np.where(s == 1, u, v))
        assert all(r == 0 for _, r in m.guard_stats())
        # slots 1, 2 hold device-to-device replicas of slot 0's converted key
        assert len({m.key_digest(i) for i in range(3)}) == 1
    finally:
        m.close()


def _shard_seams(B, world):
    idx = set()
    for r in range(world):
        lo, hi = T.shard_range(B, r, world)
        idx.update(v for v in (lo, lo + 1, hi - 2, hi - 1) if lo <= v < hi)
    return np.array(sorted(idx))


def test_multi_context_all_visible_devices(keyset, okey, rng):
    """One slot per visible GPU (slots > 0 hold peer-copied key replicas): every shard's seams
    Torus32-for-Torus32 against the exact oracle, every output against the truth table, and the
    whole batch word for word against one context on device 0."""
    torch = _torch()
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("one GPU visible: the split is covered by test_multi_context_split_bit_exact "
                    "(3 slots of device 0) and test_key_replica_bytes_and_results")
    m = T.MultiContext(keyset.bk, keyset.ksk, list(range(n)))
    one = T.Context(keyset.bk, keyset.ksk, device=0)
    try:
        B = 64 * n + 3
        x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
        host = keyset.encrypt(x, rng) + keyset.encrypt(y, rng)
        got = m.gate_host("NAND", *host)
        assert np.array_equal(keyset.decrypt(*got), 1 - (x & y))
        idx = _shard_seams(B, n)
        o = okey.gate_batch("NAND", *(v[idx] for v in host))
        bad = [int(i) for k, i in enumerate(idx) if not (np.array_equal(got[0][i], o[0][k]) and got[1][i] == o[1][k])]
        assert not bad, f"outputs differing from the oracle (Torus32) at {bad}"
        ref = one.gate_host("NAND", *host)
        assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
        assert len({m.key_digest(i) for i in range(n)}) == 1, "key replicas differ from slot 0's key"
    finally:
        one.close()
        m.close()


def test_key_replica_bytes_and_results(ctx, okey, keyset, rng):
    """tfhe_amd_context_create_replica copies a context's converted key device to device (xGMI
    peer copies between GPUs; here the last visible GPU, device 0 itself on a one-GPU box): the
    replica's key bytes equal the source's (digest of every domain) and its gates equal the
    source's word for word and the oracle's at the ends."""
    torch = _torch()
    dev = torch.cuda.device_count() - 1
    r = T.Context.replica_of(ctx, dev)
    try:
        assert r.key_digest() == ctx.key_digest()
        assert r.key_bytes() == ctx.key_bytes()
        B = 67
        x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
        host = keyset.encrypt(x, rng) + keyset.encrypt(y, rng)
        a = r.gate_host("XNOR", *host)
        b = ctx.gate_host("XNOR", *host)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
        idx = np.array([0, B - 1])
        o = okey.gate_batch("XNOR", *(v[idx] for v in host))
        assert np.array_equal(a[0][idx], o[0]) and np.array_equal(a[1][idx], o[1])
    finally:
        r.close()


def test_library_calls_keep_the_callers_current_device(keyset, rng):
    """Every entry point makes its context's device current only for the call (DeviceScope,
    engine.h): a caller working on another GPU keeps its current device, which torch and HIP
    allocate on.  On one GPU the call must leave device 0 current."""
    torch = _torch()
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("one GPU visible: no device switch to restore (DeviceScope's save/restore logic is "
                    "unit-tested on the CPU, tests/test_concurrency_tsan.py)")
    mine = n - 1   # the caller's device; the context lives on device 0
    torch.cuda.set_device(mine)
    c = T.Context(keyset.bk, keyset.ksk, device=0)
    try:
        B = 5
        x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
        got = c.gate_host("AND", *(keyset.encrypt(x, rng) + keyset.encrypt(y, rng)))
        assert np.array_equal(keyset.decrypt(*got), x & y)
        assert torch.cuda.current_device() == mine
        assert torch.empty(1, device="cuda").device.index == mine
    finally:
        c.close()
        assert torch.cuda.current_device() == mine
        torch.cuda.set_device(0)


def test_tfhe_gpu_init_and_boots_batch(ctx, keyset, rng):
    """tfhe_gpu_boots_batch before (Tier-1 device) and after tfhe_gpu_init (multi-device
    context over the visible GPUs) gives the same samples as the device context."""
    torch = _torch()
    B = 70
    x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
    host = keyset.encrypt(x, rng) + keyset.encrypt(y, rng)
    want = ctx.gate_host("ANDYN", *host)
    before = T.gpu_boots_batch(keyset.cloud, "ANDYN", *host)
    T.gpu_init(keyset.cloud, (1 << torch.cuda.device_count()) - 1)
    after = T.gpu_boots_batch(keyset.cloud, "ANDYN", *host)
    for got in (before, after):
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    assert np.array_equal(keyset.decrypt(*after), x & (1 - y))


def _slots():
    """device slots for a multi-context: every visible GPU, or two contexts on device 0"""
    n = _torch().cuda.device_count()
    return list(range(n)) if n > 1 else [0, 0]


def test_multi_gate_batch_dev_resident_shards(ctx, okey, keyset, rng):
    """tfhe_amd_multi_gate_batch_dev: each slot's shard already in its device's HBM (no PCIe in the
    loop), enqueued on every slot and synced; the shards equal one context's evaluation of the
    whole batch word for word (NAND, ragged 3 + 2 split, and MUX), the oracle on the seams."""
    torch = _torch()
    slots = _slots()
    m = T.MultiContext(keyset.bk, keyset.ksk, slots)
    try:
        for gate, B in (("NAND", 261), ("MUX", 67)):
            bits = [rng.integers(0, 2, B) for _ in range(3 if gate == "MUX" else 2)]
            host = [v for b in bits for v in keyset.encrypt(b, rng)]
            want = ctx.gate_host(gate, *host)
            shards, outs = [], []
            for i, d in enumerate(slots):
                lo, hi = T.shard_range(B, i, len(slots))
                dev = [torch.from_numpy(np.ascontiguousarray(v[lo:hi])).to(f"cuda:{d}") for v in host]
                r_a = torch.empty((hi - lo, 500), dtype=torch.int32, device=f"cuda:{d}")
                r_b = torch.empty(hi - lo, dtype=torch.int32, device=f"cuda:{d}")
                shards.append([r_a, r_b] + dev)
                outs.append((lo, hi, r_a, r_b))
            m.gate_dev(gate, shards)
            m.sync()
            got_a = np.concatenate([o[2].cpu().numpy() for o in outs])
            got_b = np.concatenate([o[3].cpu().numpy() for o in outs])
            assert np.array_equal(got_a, want[0]) and np.array_equal(got_b, want[1]), gate
            seam = np.unique([0, outs[0][1] - 1, outs[0][1], B - 1])
            o = okey.gate_batch(gate, *(v[seam] for v in host))
            assert np.array_equal(got_a[seam], o[0]) and np.array_equal(got_b[seam], o[1]), gate
    finally:
        m.close()


def _small_circuit():
    C = T.Circuit()
    a, b = C.inputs(8), C.inputs(8)
    s, co = C.add(a, b)
    gt = C.compare(a, b, "GT")
    mn = C.minmax(a, b)
    return C, a, b, s + [co, gt] + mn


def test_multi_circuit_host_and_dev_equal_one_context(ctx, keyset, rng):
    """tfhe_amd_multi_circuit_run_host / _run_dev: one circuit's instances sharded over the slots
    (here 37 instances of 8-bit add + compare + min), each slot in its own HBM wire arrays; the
    output wires equal one context's run of all 37 instances word for word, and decrypt to the
    integer results."""
    torch = _torch()
    slots = _slots()
    C, a, b, outs = _small_circuit()
    B = 37
    x, y = rng.integers(0, 256, B), rng.integers(0, 256, B)
    x[0], y[0] = 255, 255
    ins = a + b
    planes = T.bits_of(x, 8) + T.bits_of(y, 8)
    enc = [keyset.encrypt(p, rng) for p in planes]
    in_a = np.stack([e[0] for e in enc]); in_b = np.stack([e[1] for e in enc])
    n_w = C.info()["wires"]
    # one context, all instances
    wa = torch.zeros((n_w, B, 500), dtype=torch.int32, device="cuda")
    wb = torch.zeros((n_w, B), dtype=torch.int32, device="cuda")
    wa[ins] = torch.from_numpy(in_a).cuda(); wb[ins] = torch.from_numpy(in_b).cuda()
    C.run_dev(ctx, B, wa, wb)
    torch.cuda.synchronize()
    one_a, one_b = wa[outs].cpu().numpy(), wb[outs].cpu().numpy()
    m = T.MultiContext(keyset.bk, keyset.ksk, slots)
    try:
        got_a, got_b = m.circuit_host(C, B, ins, in_a, in_b, outs)
        assert np.array_equal(got_a, one_a) and np.array_equal(got_b, one_b)
        shards = []
        for i, d in enumerate(slots):
            lo, hi = T.shard_range(B, i, len(slots))
            sa = torch.zeros((n_w, hi - lo, 500), dtype=torch.int32, device=f"cuda:{d}")
            sb = torch.zeros((n_w, hi - lo), dtype=torch.int32, device=f"cuda:{d}")
            sa[ins] = torch.from_numpy(np.ascontiguousarray(in_a[:, lo:hi])).to(sa.device)
            sb[ins] = torch.from_numpy(np.ascontiguousarray(in_b[:, lo:hi])).to(sb.device)
            shards.append((sa, sb))
        m.circuit_dev(C, shards)
        m.sync()
        dev_a = np.concatenate([sh[0][outs].cpu().numpy() for sh in shards], axis=1)
        dev_b = np.concatenate([sh[1][outs].cpu().numpy() for sh in shards], axis=1)
        assert np.array_equal(dev_a, one_a) and np.array_equal(dev_b, one_b)
    finally:
        m.close()
    dec = [keyset.decrypt(got_a[k], got_b[k]) for k in range(len(outs))]
    assert np.array_equal(T.int_of(dec[:9]), x + y)
    assert np.array_equal(dec[9], (x > y).astype(np.int64))
    assert np.array_equal(T.int_of(dec[10:]), np.minimum(x, y))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_on_gpu(rank, world, port, q):
    import torch.distributed as dist
    import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    K = T.SecretKeyset()
    c = T.Context(K.bk, K.ksk, device=0)          # every rank's replica (one GPU on this box)
    inputs = None
    if rank == 0:
        rng = np.random.default_rng(5)
        B = 257
        x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
        inputs = K.encrypt(x, rng) + K.encrypt(y, rng)
    out = D.run_sharded(lambda a_a, a_b, b_a, b_b: c.gate_host("NAND", a_a, a_b, b_a, b_b), inputs, rank, world)
    if rank == 0:
        okey = O.OracleKey(K.bk, K.ksk)
        idx = np.array([0, 128, 129, 256])
        o = okey.gate_batch("NAND", *(v[idx] for v in inputs))
        single = c.gate_host("NAND", *inputs)
        q.put((np.array_equal(out[0], single[0]) and np.array_equal(out[1], single[1]),
               np.array_equal(out[0][idx], o[0]) and np.array_equal(out[1][idx], o[1])))
    dist.barrier()
    c.close()
    K.close()
    dist.destroy_process_group()


def test_two_ranks_scatter_gpu_gather():
    """torchrun's shape on one card: two ranks, rank 0 scatters 257 gates (129 + 128), each
    rank evaluates its shard on its own GPU context, rank 0 gathers: the same samples as one
    context's evaluation of the whole batch, and the oracle's at the seam."""
    world = 2
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_rank_on_gpu, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    same, exact = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert same and exact


def test_multi_and_mixed_edge_cases(ctx, okey, keyset, rng):
    """Edge shapes of the round-3 APIs: a device-resident multi batch whose second slot is empty, a
    one-instance circuit over two slots (one idles), B = 0 everywhere, and mixed batches of a single
    gate and of MUX only — all equal to the single-context path / the oracle."""
    torch = _torch()
    m = T.MultiContext(keyset.bk, keyset.ksk, [0, 0])
    try:
        B = 5
        x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
        host = keyset.encrypt(x, rng) + keyset.encrypt(y, rng)
        dev = [torch.from_numpy(v).cuda() for v in host]
        r_a = torch.empty((B, 500), dtype=torch.int32, device="cuda")
        r_b = torch.empty(B, dtype=torch.int32, device="cuda")
        empty = [torch.empty((0, 500), dtype=torch.int32, device="cuda"), torch.empty(0, dtype=torch.int32, device="cuda")] * 3
        m.gate_dev("AND", [[r_a, r_b] + dev, empty])
        m.sync()
        want = ctx.gate_host("AND", *host)
        assert np.array_equal(r_a.cpu().numpy(), want[0]) and np.array_equal(r_b.cpu().numpy(), want[1])
        m.gate_dev("AND", [empty, empty])                       # B = 0 on both slots
        m.sync()
        C = T.Circuit()
        a, b = C.inputs(4), C.inputs(4)
        s, co = C.add(a, b)
        planes = T.bits_of(np.array([9]), 4) + T.bits_of(np.array([7]), 4)
        enc = [keyset.encrypt(p, rng) for p in planes]
        out_a, out_b = m.circuit_host(C, 1, a + b, np.stack([e[0] for e in enc]), np.stack([e[1] for e in enc]),
                                      s + [co])
        assert T.int_of([keyset.decrypt(out_a[k], out_b[k]) for k in range(5)])[0] == 16
        z = np.zeros((0, 0, 500), np.int32)
        m.circuit_host(C, 0, [], z, np.zeros((0, 0), np.int32), [])
    finally:
        m.close()
    (sa, sb), (ua, ub), (va, vb) = (keyset.encrypt(rng.integers(0, 2, 3), rng) for _ in range(3))
    got = ctx.gate_mixed_host(["MUX"] * 3, sa, sb, ua, ub, va, vb)
    want = okey.gate_batch("MUX", sa, sb, ua, ub, va, vb)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    got1 = ctx.gate_mixed_host(["XNOR"], sa[:1], sb[:1], ua[:1], ub[:1])
    want1 = okey.gate_batch("XNOR", sa[:1], sb[:1], ua[:1], ub[:1])
    assert np.array_equal(got1[0], want1[0]) and np.array_equal(got1[1], want1[1])


def test_bench_multi_device_leg_child_process():
    """bench.py's one-process multi-device leg runs in a child process under a time limit (a fault
    on a many-GPU host costs that leg, not the headline line): rehearsed here with two slots on
    device 0, the child reports a rate and a correct NAND truth table on every shard."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--multi-only", "--multi-devices", "0,0",
                        "--batch", "96", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stderr[-2000:])
    out = json.loads(lines[-1])
    assert out.get("devices") == 2 and out["truth_table_ok"] is True and out["value"] > 0, out
