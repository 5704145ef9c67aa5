"""Encrypted matrix-vector product sharded over GPUs (BASELINE config 5).

y = A x for an R x C matrix A and a C-vector x of unsigned `nbits` integers, all encrypted
bit by bit.  The reference multiplies all element pairs (BOOTS_vectorMultiplication) and
folds the products with a tree of ripple adders (BOOTS_matrixMultiplication,
gpuParallel/main.cu:2342-2462; Cannon's algorithm :2590-2645) on one GPU.  Here:

* one circuit computes ONE output element: `Circuit.dot` puts every partial product of the C
  terms into a single Dadda tree (csrc/circuit.cpp), depth ~25 for C = 64, nbits = 16;
* the circuit's instance dimension is the matrix row: a rank evaluates its rows as the B
  instances of that circuit, so every level is one launch over (gates x rows);
* rows are sharded contiguously over ranks (shard.shard_range); rows are independent, so
  there is no collective on the data path — each rank decrypts / checks its own rows and only
  the timing is reduced (max over ranks).  Keys are replicated per GPU;
* or, from ONE host process: `run_rows_multi` hands all rows to the library's multi-device
  circuit run (tfhe_amd_multi_circuit_run_host, csrc/multi.cpp), which shards them over the
  devices of a MultiContext (one worker thread and key replica per device), the way a C++ host
  such as the reference's cloud.cpp would drive a node.
"""
import numpy as np

import shard


def out_bits(cols, nbits):
    return 2 * nbits + int(np.ceil(np.log2(max(cols, 2))))


def build(T, cols, nbits):
    """circuit for one output element: (circuit, a wires [cols][nbits], x wires, y wires)"""
    C = T.Circuit()
    a = [C.inputs(nbits) for _ in range(cols)]
    x = [C.inputs(nbits) for _ in range(cols)]
    y = C.dot(a, x, out_bits(cols, nbits))
    return C, a, x, y


def shard_rows(rows, rank, world):
    return shard.shard_range(rows, rank, world)


def instance_inputs(T, a_wires, x_wires, A_rows, x_vec, nbits):
    """{wire: bit plane over the instances} for the rows A_rows ([B][cols]) and vector x."""
    bits = {}
    B = A_rows.shape[0]
    for t in range(A_rows.shape[1]):
        bits.update(zip(a_wires[t], T.bits_of(A_rows[:, t], nbits)))
        bits.update(zip(x_wires[t], T.bits_of(np.full(B, x_vec[t]), nbits)))
    return bits


def run_rows_gpu(T, torch, ctx, keyset, C, a_w, x_w, y_w, A_rows, x_vec, nbits, rng, reps=1, barrier=None):
    """Encrypt this rank's rows, evaluate on the GPU, decrypt: (y [B], seconds per run)."""
    import time
    B = A_rows.shape[0]
    n_w = C.info()["wires"]
    wa = torch.zeros((n_w, B, 500), dtype=torch.int32, device="cuda")
    wb = torch.zeros((n_w, B), dtype=torch.int32, device="cuda")
    for w, plane in instance_inputs(T, a_w, x_w, A_rows, x_vec, nbits).items():
        ea, eb = keyset.encrypt(plane, rng)
        wa[w] = torch.from_numpy(ea).cuda()
        wb[w] = torch.from_numpy(eb).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    C.run_dev(ctx, B, wa, wb, stream)                      # warm-up: compile + table upload
    times = []
    for _ in range(reps):
        torch.cuda.synchronize()
        if barrier:
            barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        C.run_dev(ctx, B, wa, wb, stream)
        torch.cuda.synchronize()
        if barrier:
            barrier()
        times.append(time.perf_counter() - t0)
    ha, hb = wa.cpu().numpy(), wb.cpu().numpy()
    y = T.int_of([keyset.decrypt(ha[w], hb[w]) for w in y_w])
    return y, float(np.median(times))


def encrypt_inputs(T, keyset, a_wires, x_wires, A_rows, x_vec, nbits, rng):
    """(input wire ids, in_a [n_in][B][500], in_b [n_in][B]) for the multi-device host API"""
    bits = instance_inputs(T, a_wires, x_wires, A_rows, x_vec, nbits)
    wires = sorted(bits)
    B = A_rows.shape[0]
    in_a = np.empty((len(wires), B, 500), np.int32)
    in_b = np.empty((len(wires), B), np.int32)
    for k, w in enumerate(wires):
        in_a[k], in_b[k] = keyset.encrypt(bits[w], rng)
    return wires, in_a, in_b


def run_rows_multi(T, multi, keyset, C, a_w, x_w, y_w, A_rows, x_vec, nbits, rng, extra_out=()):
    """All rows through one MultiContext (rows sharded over its device slots inside the library):
    (y [B], seconds, {wire: (a [B][500], b [B])} for the extra output wires, the encrypted inputs)."""
    import time
    wires, in_a, in_b = encrypt_inputs(T, keyset, a_w, x_w, A_rows, x_vec, nbits, rng)
    outs = list(y_w) + list(extra_out)
    B = A_rows.shape[0]
    t0 = time.perf_counter()
    out_a, out_b = multi.circuit_host(C, B, wires, in_a, in_b, outs)
    dt = time.perf_counter() - t0
    y = T.int_of([keyset.decrypt(out_a[k], out_b[k]) for k in range(len(y_w))])
    extra = {w: (out_a[len(y_w) + k], out_b[len(y_w) + k]) for k, w in enumerate(extra_out)}
    return y, dt, extra, (wires, in_a, in_b)
