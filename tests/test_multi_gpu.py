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
    finally:
        m.close()


def test_multi_context_all_visible_devices(keyset, rng):
    torch = _torch()
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("one GPU visible: the split is covered by test_multi_context_split_bit_exact")
    m = T.MultiContext(keyset.bk, keyset.ksk, list(range(n)))
    try:
        B = 64 * n + 3
        x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
        got = m.gate_host("NAND", *(keyset.encrypt(x, rng) + keyset.encrypt(y, rng)))
        assert np.array_equal(keyset.decrypt(*got), 1 - (x & y))
    finally:
        m.close()


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
