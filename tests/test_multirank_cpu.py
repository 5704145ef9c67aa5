"""N>1 path on CPU: gloo, world_size 2 — shard ranges partition the batch and the timing
reduction returns the max over ranks (the only collective; none on the data path)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard.shard_range(1000, rank, world)
    elapsed = 1.0 + rank            # rank 1 is the slow one
    m = shard.max_over_ranks(elapsed)
    out.put((rank, lo, hi, m))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_sharding_and_timing():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1:3] for r in res] == [(0, 500), (500, 1000)]
    assert all(r[3] == 2.0 for r in res)
    assert shard.weak_scaling_value(1024, 2, 5, 2.0) == 1024 * 2 * 5 / 2.0


@pytest.mark.parametrize("total,world", [(0, 3), (7, 3), (1024, 8), (4096, 8), (5, 8)])
def test_shards_partition(total, world):
    spans = [shard.shard_range(total, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    sizes = [hi - lo for lo, hi in spans]
    assert max(sizes) - min(sizes) <= 1


def test_max_over_ranks_identity_single_process():
    assert shard.max_over_ranks(3.5) == 3.5


def _matvec_worker(rank, world, port, out):
    """each rank evaluates its row shard of a small encrypted-style matrix-vector product in
    plaintext (the engine's own torus arithmetic, Circuit.eval_plain); rows are gathered only
    to check the result here — the product path itself has no collective."""
    import numpy as np
    import torch.distributed as dist
    import matvec
    import tfhe_amd as T
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(11)
    rows, cols, nbits = 5, 4, 3
    A = rng.integers(0, 2**nbits, (rows, cols))
    x = rng.integers(0, 2**nbits, cols)
    lo, hi = matvec.shard_rows(rows, rank, world)
    C, a_w, x_w, y_w = matvec.build(T, cols, nbits)
    val = C.eval_plain(matvec.instance_inputs(T, a_w, x_w, A[lo:hi], x, nbits))
    y = T.int_of([val[w] for w in y_w])
    got = [None] * world
    dist.all_gather_object(got, (lo, hi, [int(v) for v in np.atleast_1d(y)]))
    out.put((rank, got, [int(v) for v in A @ x]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_matvec_shards():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_matvec_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, got, want in res:
        full = []
        for lo, hi, ys in sorted(got):
            assert len(ys) == hi - lo
            full += ys
        assert full == want
