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


def test_library_shard_range_matches_python():
    """The library's multi-device split (tfhe_amd_shard_range) is shard.py's arithmetic."""
    import tfhe_amd as T
    for total in (0, 1, 5, 7, 1000, 1024, 4096, 4097):
        for world in (1, 2, 3, 4, 8):
            for r in range(world):
                assert T.shard_range(total, r, world) == shard.shard_range(total, r, world)


def _driver_worker(rank, world, port, q):
    """one rank of the real driver path: rank 0 holds the batch, dist.run_sharded scatters it,
    every rank evaluates its shard (here on the CPU oracle: the per-rank GPU context is the
    same call on the box), rank 0 gathers."""
    import numpy as np
    import torch.distributed as dist
    import dist as D
    import oracle_ctypes as O
    import tfhe_amd as T
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    K = T.SecretKeyset()                      # the same seeded key on every rank (replicas)
    okey = O.OracleKey(K.bk, K.ksk)
    inputs = None
    if rank == 0:
        rng = np.random.default_rng(77)
        B = 5
        x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
        inputs = K.encrypt(x, rng) + K.encrypt(y, rng)
    evaluated = []

    def evaluate(a_a, a_b, b_a, b_b):
        evaluated.append(a_a.shape[0])
        return okey.gate_batch("NAND", a_a, a_b, b_a, b_b, nthreads=2)
    out = D.run_sharded(evaluate, inputs, rank, world)
    if rank == 0:
        want = okey.gate_batch("NAND", *inputs, nthreads=2)
        ok = np.array_equal(out[0], want[0]) and np.array_equal(out[1], want[1])
        truth = np.array_equal(K.decrypt(*out), 1 - (K.decrypt(*inputs[:2]) & K.decrypt(*inputs[2:])))
        q.put((rank, evaluated, ok, truth))
    else:
        q.put((rank, evaluated, None, None))
    dist.barrier()
    dist.destroy_process_group()
    K.close()


def test_two_rank_gloo_scatter_evaluate_gather():
    """world_size 2 over gloo: a ragged batch of 5 gates is scattered (3 + 2), evaluated per rank
    and gathered; the gathered Torus32 outputs equal one process's evaluation of the whole batch
    word for word and decrypt to the NAND truth table."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_driver_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == [3] and res[1][1] == [2]          # contiguous shards of 5 over 2 ranks
    assert res[0][2] is True and res[0][3] is True


def _matmat_worker(rank, world, port, out):
    """each rank evaluates its block of output rows of C = A B (plaintext, the engine's own
    torus arithmetic); blocks are gathered here only to check the whole product."""
    import numpy as np
    import torch.distributed as dist
    import matmat
    import tfhe_amd as T
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(13)
    m, k, n, nbits = 5, 3, 4, 4
    A = rng.integers(0, 2**nbits, (m, k))
    Bm = rng.integers(0, 2**nbits, (k, n))
    lo, hi = matmat.shard_rows(m, rank, world)
    C, a_w, b_w, c_w = matmat.build(T, k, nbits)
    val = C.eval_plain(matmat.instance_inputs(T, a_w, b_w, A[lo:hi], Bm, nbits))
    blk = np.asarray(T.int_of([val[w] for w in c_w])).reshape(hi - lo, n)
    got = [None] * world
    dist.all_gather_object(got, (lo, hi, blk.tolist()))
    out.put((rank, got, ((A @ Bm) % 2**nbits).tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_matmat_row_blocks():
    """C = A B mod 2^nbits (the reference's single-precision BOOTS_matrixMultiplication) with
    row blocks of C on two gloo ranks: the blocks assemble to the integer product."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_matmat_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, got, want in res:
        full = []
        for lo, hi, blk in sorted(got):
            assert len(blk) == hi - lo
            full += blk
        assert full == want


def _ranks_worker(rank, world, port, mode, out):
    """bench.rank_block over gloo with the device identity stubbed (no GPU here): every rank's
    record is gathered; devices count as distinct by PCI function or, failing that, by UUID (a
    partitioned part's logical GPUs share a PCI function); a shared device is reported (a warning
    under RCCL), never raised."""
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = 0 if mode == "same" else rank
    pci = 0x10 if mode != "distinct" else 0x10 + dev
    bench.device_identity = lambda torch, local: {"device": dev, "name": "stub", "cus": 256,
                                                  "pci": "0000:%02x:00" % pci, "uuid": "GPU-%d" % dev}
    parity = {"checked_per_rank": 128, "mismatches": 0, "mismatches_local": rank}
    strong_ok = {"1024": rank == 0, "4096": True}
    blk = bench.rank_block(dist, None, rank, "gloo", rank, world, True, parity, strong_ok, 3.0 + rank)
    blk_nccl = bench.rank_block(dist, None, rank, "nccl", rank, world, True, parity, strong_ok, 3.0)
    out.put((rank, blk, blk_nccl["distinct_devices"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["distinct", "same", "partitioned"])
def test_two_rank_bench_ranks_block(mode):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ranks_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, blk, distinct_nccl in res:
        assert blk["world_size"] == 2 and blk["backend"] == "gloo"
        assert [r["rank"] for r in blk["per_rank"]] == [0, 1]
        assert [r["parity_mismatches_local"] for r in blk["per_rank"]] == [0, 1]
        assert [r["strong_truth_table_ok"]["1024"] for r in blk["per_rank"]] == [True, False]
        assert [r["strong_truth_table_ok"]["4096"] for r in blk["per_rank"]] == [True, True]
        assert blk["distinct_devices"] == (mode != "same") == distinct_nccl
