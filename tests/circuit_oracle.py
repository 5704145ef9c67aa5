"""Node-by-node CPU evaluation of a circuit (include/tfhe_amd.h) with the exact oracle's bootstraps
(TEST INFRASTRUCTURE: used by tests/test_configs_gpu.py as the checker of whole circuits).

The GPU compiles a circuit into level-batched rows in which bootstrap-free nodes (NOT, COPY,
CONST) are folded into the rows that read them; this evaluator does NOT fold: it walks the nodes
in SSA order, materialises every wire as an LWE sample and bootstraps each gate node from the
linear combination of its input wires, exactly as the reference evaluates gates one by one:
  * gate / lincomb node:  W = lweKeySwitch(woKS(mu = 1/8, (0, c0) + sum_k s_k W[in_k]))
    (boot-gates.cu:98-397: the prologue constants and signs of tfhe_amd_circuit_gate's rows);
  * MUX node:             W = lweKeySwitch((0, 1/8) + woKS(-1/8 + a + b) + woKS(-1/8 - a + c))
    (boot-gates.cu:407-448);
  * NOT / COPY / CONST:   W = -W[in], W[in], (0, c0) (boot-gates.cu:242-267).
Integer arithmetic mod 2^32 throughout, so folding (the GPU's) and not folding (here) must give
the same Torus32 words — the comparison checks the compiler's folding and the row kernels at once.
Gates of one bootstrap depth are batched into one oracle call per depth."""
import numpy as np

E8 = 1 << 29
MUX = 10


def _wrap(x):
    return ((np.asarray(x, dtype=np.int64) + 2**31) % 2**32 - 2**31).astype(np.int32)


def eval_circuit(C, okey, inputs, B, nthreads=0):
    """C: tfhe_amd.Circuit; inputs: {wire: (a [B][500] int32, b [B] int32)};
    returns {wire: (a, b)} for every wire."""
    n_w = C.info()["wires"]
    nodes = [C.node(w) for w in range(n_w)]
    W = {}
    depth = {}
    for w, (kind, gate, c0, s, ins) in enumerate(nodes):
        if kind == 0:
            W[w] = tuple(np.asarray(v, dtype=np.int32) for v in inputs[w])
            depth[w] = 0
        elif kind == 2:
            depth[w] = depth[ins[0]] if ins[0] >= 0 else 0
        else:
            depth[w] = 1 + max(depth[i] for i in ins if i >= 0)
    max_d = max(depth.values()) if depth else 0

    def lin(c, terms):
        a = np.zeros((B, 500), np.int64)
        b = np.full(B, c, np.int64)
        for sk, wk in terms:
            a += np.int64(sk) * W[wk][0].astype(np.int64)
            b += np.int64(sk) * W[wk][1].astype(np.int64)
        return _wrap(a), _wrap(b)

    for d in range(max_d + 1):
        # affine nodes whose input is ready (in SSA order, so chains resolve)
        todo_rows, todo_meta = [], []
        for w, (kind, gate, c0, s, ins) in enumerate(nodes):
            if depth[w] != d or kind == 0:
                continue
            if kind == 2:
                continue
            if gate == MUX:
                r1 = lin(-E8, [(1, ins[0]), (1, ins[1])])
                r2 = lin(-E8, [(-1, ins[0]), (1, ins[2])])
                todo_meta.append((w, True, len(todo_rows)))
                todo_rows += [r1, r2]
            else:
                r = lin(c0, [(s[k], ins[k]) for k in range(3) if ins[k] >= 0 and s[k] != 0])
                todo_meta.append((w, False, len(todo_rows)))
                todo_rows.append(r)
        if todo_rows:
            xa = np.concatenate([r[0] for r in todo_rows])
            xb = np.concatenate([r[1] for r in todo_rows])
            ua, ub = okey.woks_batch(E8, xa, xb, nthreads=nthreads)
            ks_a, ks_b = [], []
            for w, mux, k in todo_meta:
                sa, sb = ua[k * B:(k + 1) * B], ub[k * B:(k + 1) * B]
                if mux:
                    sa = _wrap(sa.astype(np.int64) + ua[(k + 1) * B:(k + 2) * B])
                    sb = _wrap(sb.astype(np.int64) + ub[(k + 1) * B:(k + 2) * B] + E8)
                ks_a.append(sa)
                ks_b.append(sb)
            ra, rb = okey.keyswitch_batch(np.concatenate(ks_a), np.concatenate(ks_b), nthreads=nthreads)
            for j, (w, _, _) in enumerate(todo_meta):
                W[w] = (ra[j * B:(j + 1) * B], rb[j * B:(j + 1) * B])
        for w, (kind, gate, c0, s, ins) in enumerate(nodes):
            if depth[w] == d and kind == 2:
                if gate == 15:                                   # CONST
                    W[w] = (np.zeros((B, 500), np.int32), np.full(B, c0, np.int32))
                elif gate == 13:                                 # NOT
                    W[w] = (_wrap(-W[ins[0]][0].astype(np.int64)), _wrap(-W[ins[0]][1].astype(np.int64)))
                else:                                            # COPY
                    W[w] = (W[ins[0]][0].copy(), W[ins[0]][1].copy())
    return W
