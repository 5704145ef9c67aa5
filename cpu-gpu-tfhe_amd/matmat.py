"""Encrypted matrix x matrix product sharded over GPUs.

C = A B for an m x k matrix A and a k x n matrix B of unsigned `nbits` integers, encrypted bit
by bit.  The reference multiplies every element pair of the two matrices (BOOTS_vectorMultiplication
over row * col * row pairs) and folds them with vector additions (BOOTS_matrixMultiplication,
gpuParallel/main.cu:2342-2462), or rotates the operands k times in Cannon's algorithm
(BOOTS_CannonsAlgo, main.cu:2590-2645; layout helpers matrixUtility.cu:65-96), all on one GPU;
by default (isDoublePrecision = false) the result keeps nbits bits, i.e. C mod 2^nbits.

Here:
* one circuit computes ONE output element, the dot product of a row of A and a column of B:
  `Circuit.dot` puts all k * nbits^2 partial products below the output width into a single
  Dadda tree (csrc/circuit.cpp), so there is no separate multiply / add stage per pair;
* the circuit's instance dimension is the output element (i, j): a rank evaluates its block of
  output rows (rows_lo .. rows_hi) x all n columns as the B = rows x n instances of that one
  circuit, so every level is one launch over (gates x elements);
* row blocks are sharded contiguously over ranks (shard.shard_range); blocks are independent,
  no collective on the data path (keys replicated, A's row block and all of B per rank).
"""
import numpy as np

import shard


def out_bits(k, nbits, double_precision=False):
    return 2 * nbits + int(np.ceil(np.log2(max(k, 2)))) if double_precision else nbits


def build(T, k, nbits, double_precision=False):
    """circuit for one output element: (circuit, a wires [k][nbits], b wires [k][nbits], c wires)"""
    C = T.Circuit()
    a = [C.inputs(nbits) for _ in range(k)]
    b = [C.inputs(nbits) for _ in range(k)]
    c = C.dot(a, b, out_bits(k, nbits, double_precision))
    return C, a, b, c


def shard_rows(m, rank, world):
    return shard.shard_range(m, rank, world)


def instance_inputs(T, a_wires, b_wires, A_rows, Bm, nbits):
    """{wire: bit plane over the instances (i, j), row-major} for the row block A_rows
    ([r][k]) against all columns of B ([k][n])."""
    r, k = A_rows.shape
    n = Bm.shape[1]
    bits = {}
    for t in range(k):
        av = np.repeat(A_rows[:, t], n)             # instance (i, j) -> A[i][t]
        bv = np.tile(Bm[t, :], r)                   # instance (i, j) -> B[t][j]
        bits.update(zip(a_wires[t], T.bits_of(av, nbits)))
        bits.update(zip(b_wires[t], T.bits_of(bv, nbits)))
    return bits


def run_block_gpu(T, torch, ctx, keyset, C, a_w, b_w, c_w, A_rows, Bm, nbits, rng, reps=1, barrier=None):
    """Encrypt this rank's row block, evaluate on the GPU, decrypt: (C block [r][n], s per run)."""
    import time
    r, n = A_rows.shape[0], Bm.shape[1]
    inst = r * n
    n_w = C.info()["wires"]
    wa = torch.zeros((n_w, inst, 500), dtype=torch.int32, device="cuda")
    wb = torch.zeros((n_w, inst), dtype=torch.int32, device="cuda")
    for w, plane in instance_inputs(T, a_w, b_w, A_rows, Bm, nbits).items():
        ea, eb = keyset.encrypt(plane, rng)
        wa[w] = torch.from_numpy(ea).cuda()
        wb[w] = torch.from_numpy(eb).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    C.run_dev(ctx, inst, wa, wb, stream)                 # warm-up: compile + table upload
    times = []
    for _ in range(reps):
        torch.cuda.synchronize()
        if barrier:
            barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        C.run_dev(ctx, inst, wa, wb, stream)
        torch.cuda.synchronize()
        if barrier:
            barrier()
        times.append(time.perf_counter() - t0)
    ha, hb = wa.cpu().numpy(), wb.cpu().numpy()
    c = T.int_of([keyset.decrypt(ha[w], hb[w]) for w in c_w])
    return np.asarray(c).reshape(r, n), float(np.median(times))
