// circuit.cpp — batched circuit schedules over the MI355X engine.
//
// The reference evaluates Cipher's integer operations (cpuParallel/Cipher.cpp:83-392) one
// synchronous gate at a time, and its GPU path batches hand-written gate groups
// (taskLevelParallelAdd_bitwise gpuParallel/main.cu:821-890, the compound ANDXOR / XORXOR
// gates boot-gates.cu:3027-3098, multiplyLweSamples main.cu:1483-1579).  Here a circuit is a
// DAG of gates over SSA wires; the compiler levels it by bootstrap depth and every level runs
// as ONE blind-rotation launch over all of its gates x B independent instances plus ONE key
// switch launch, so any circuit gets the batching the reference wrote by hand for two.
//
// Bootstrap-free gates (NOT, COPY, CONSTANT; boot-gates.cu:242-267) become affine forms
// (0, c) + s W[base] that are folded into the rows that consume them and also materialised
// in the wire array.  Three-input rows give MAJ and XOR3 in one bootstrap each, so a
// full adder is one level (2 bootstraps) instead of the reference's three (5 bootstraps).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "engine.h"
#include "../../include/tfhe_amd.h"
#include "api_internal.h"

using namespace tfhe_amd;

namespace {

constexpr int32_t kE8 = 1 << 29;   // modSwitchToTorus32(1, 8)
constexpr int32_t kE4 = 1 << 30;   // modSwitchToTorus32(1, 4)

struct Node {
    int kind;            // 0 = input, 1 = bootstrapped row(s), 2 = affine (no bootstrap)
    int gate;            // TFHE_GATE_* (kind 1, 2) or -1
    int32_t c0;          // lincomb / affine constant
    int32_t s[3];        // lincomb coefficients
    int in[3];           // input wires (-1 = absent)
};

struct Affine {          // W = (0, c) + s W[base]; base = -1: the trivial sample (0, c)
    int32_t c, s;
    int base;
};

}  // namespace

// Device state of a circuit for ONE executing context: the level tables on its device and the
// extracted-sample scratch.  Contexts that run the same circuit at the same time (the shards of a
// multi-device run, tfhe_amd_multi_circuit_run_*; several contexts on one GPU) each get their own.
struct CircuitDevState {
    int dev = -1;
    void *d_tab = nullptr;
    int32_t *u_a = nullptr, *u_b = nullptr;
    uint32_t *u_flags = nullptr;   // exactness-guard flags, 2 words per u slot (engine.h Guard)
    size_t u_slots = 0;
    StreamFence fence;   // u scratch reuse across caller streams
    ~CircuitDevState() { release(); }
    void release() {
        DeviceScope dev_scope(dev);   // the frees below are on dev; the caller keeps its device
        if (dev >= 0) (void)hipDeviceSynchronize();   // a run on a caller's stream may still read them
        fence.release();
        if (d_tab) (void)hipFree(d_tab);
        if (u_a) (void)hipFree(u_a);
        if (u_b) (void)hipFree(u_b);
        if (u_flags) (void)hipFree(u_flags);
        d_tab = nullptr; u_a = nullptr; u_b = nullptr; u_flags = nullptr; u_slots = 0; dev = -1;
    }
};

struct TfheAmdCircuit {
    std::vector<Node> nodes;           // one per wire
    // compiled schedule
    bool compiled = false;
    struct Level { int row0, nrows, ks0, nks, lin0, nlin; };
    std::vector<Level> levels;         // levels[0]: affine nodes over inputs only
    std::vector<CircRow> rows;
    std::vector<CircKs> ks;
    std::vector<CircLin> lin;
    int n_boot = 0, max_rows = 0;
    // per executing context (keyed by the context): device tables + scratch
    std::mutex mu;   // compile + the state map; runs on distinct contexts proceed concurrently
    // keyed by the context's uid (engine.cpp; never reused), dropped when the context is destroyed
    std::unordered_map<uint64_t, std::unique_ptr<CircuitDevState>> states;
};

namespace {
// every live circuit, so that a context's destruction can drop its states (lock order: this
// registry, then a circuit's mu)
std::mutex g_circuits_mu;
std::unordered_set<TfheAmdCircuit *> g_circuits;
}  // namespace

void tfhe_amd_internal_circuits_forget_context(unsigned long long ctx_uid) {
    std::vector<std::unique_ptr<CircuitDevState>> dead;
    {
        std::lock_guard<std::mutex> reg(g_circuits_mu);
        for (TfheAmdCircuit *c : g_circuits) {
            std::lock_guard<std::mutex> lk(c->mu);
            auto it = c->states.find((uint64_t)ctx_uid);
            if (it == c->states.end()) continue;
            dead.push_back(std::move(it->second));
            c->states.erase(it);
        }
    }
    dead.clear();   // frees the device memory (CircuitDevState::release) outside the locks
}

namespace {

bool row_spec(int gate, int32_t *c, int32_t *s0, int32_t *s1, int32_t *s2) {
    // boot-gates.cu:98-397 constants; MAJ / XOR3: circuit rows of this engine
    *s2 = 0;
    switch (gate) {
    case TFHE_GATE_NAND:  *c = kE8;  *s0 = -1; *s1 = -1; return true;
    case TFHE_GATE_OR:    *c = kE8;  *s0 = 1;  *s1 = 1;  return true;
    case TFHE_GATE_AND:   *c = -kE8; *s0 = 1;  *s1 = 1;  return true;
    case TFHE_GATE_XOR:   *c = kE4;  *s0 = 2;  *s1 = 2;  return true;
    case TFHE_GATE_XNOR:  *c = -kE4; *s0 = -2; *s1 = -2; return true;
    case TFHE_GATE_NOR:   *c = -kE8; *s0 = -1; *s1 = -1; return true;
    case TFHE_GATE_ANDNY: *c = -kE8; *s0 = -1; *s1 = 1;  return true;
    case TFHE_GATE_ANDYN: *c = -kE8; *s0 = 1;  *s1 = -1; return true;
    case TFHE_GATE_ORNY:  *c = kE8;  *s0 = -1; *s1 = 1;  return true;
    case TFHE_GATE_ORYN:  *c = kE8;  *s0 = 1;  *s1 = -1; return true;
    // majority: a + b + c in {+-1/8, +-3/8}, positive iff at least two inputs are 1
    case TFHE_GATE_MAJ:   *c = 0;    *s0 = 1;  *s1 = 1;  *s2 = 1; return true;
    // parity: 2(a + b + c) is -1/4 (mod 1) for an odd number of ones and +1/4 for an even one
    case TFHE_GATE_XOR3:  *c = 0;    *s0 = -2; *s1 = -2; *s2 = -2; return true;
    default: return false;
    }
}

int n_inputs(int gate) {
    switch (gate) {
    case TFHE_GATE_MUX: case TFHE_GATE_MAJ: case TFHE_GATE_XOR3: return 3;
    case TFHE_GATE_NOT: case TFHE_GATE_COPY: return 1;
    case TFHE_GATE_CONST: return 0;
    default: return 2;
    }
}

// row = (0, c0) + sum_t coef_t * A_t with A_t affine: fold constants, merge equal bases
bool build_row(int32_t c0, const int32_t *coef, const Affine *A, int n, CircRow *row) {
    int32_t c = c0;
    int base[3] = {-1, -1, -1};
    int32_t s[3] = {0, 0, 0};
    int m = 0;
    for (int t = 0; t < n; ++t) {
        if (coef[t] == 0) continue;
        c = (int32_t)((uint32_t)c + (uint32_t)coef[t] * (uint32_t)A[t].c);
        if (A[t].base < 0 || A[t].s == 0) continue;
        const int32_t k = (int32_t)((uint32_t)coef[t] * (uint32_t)A[t].s);
        int u = 0;
        while (u < m && base[u] != A[t].base) ++u;
        if (u == m) { base[m] = A[t].base; s[m] = 0; ++m; }
        s[u] = (int32_t)((uint32_t)s[u] + (uint32_t)k);
    }
    *row = CircRow{c, s[0], s[1], s[2], base[0], base[1], base[2], 0};
    return true;
}

int compile(TfheAmdCircuit *C) {
    const int W = (int)C->nodes.size();
    std::vector<Affine> aff(W);
    std::vector<int> level(W, 0);
    // per level buckets (index 0 = affine over inputs / constants only)
    std::vector<std::vector<CircRow>> rows;
    std::vector<std::vector<CircKs>> kss;
    std::vector<std::vector<CircLin>> lins;
    auto ensure = [&](int L) {
        if ((int)rows.size() <= L) { rows.resize(L + 1); kss.resize(L + 1); lins.resize(L + 1); }
    };
    ensure(0);
    C->n_boot = 0;
    for (int w = 0; w < W; ++w) {
        const Node &nd = C->nodes[w];
        if (nd.kind == 0) { aff[w] = Affine{0, 1, w}; level[w] = 0; continue; }
        for (int t = 0; t < 3; ++t)
            if (nd.in[t] >= w) return TFHE_AMD_E_ARG;       // SSA order: inputs defined earlier
        if (nd.kind == 2) {
            Affine a;
            if (nd.gate == TFHE_GATE_CONST) a = Affine{nd.c0, 0, -1};
            else {
                const Affine &x = aff[nd.in[0]];
                const int32_t sg = nd.gate == TFHE_GATE_NOT ? -1 : 1;
                a = Affine{(int32_t)((uint32_t)sg * (uint32_t)x.c), (int32_t)((uint32_t)sg * (uint32_t)x.s), x.base};
            }
            aff[w] = a;
            level[w] = a.base < 0 ? 0 : level[a.base];
            ensure(level[w]);
            lins[level[w]].push_back(CircLin{a.c, a.s, a.base, w});
            continue;
        }
        // bootstrapped
        Affine A[3];
        int L = 0;
        for (int t = 0; t < 3; ++t) {
            if (nd.in[t] < 0) { A[t] = Affine{0, 0, -1}; continue; }
            A[t] = aff[nd.in[t]];
            if (A[t].base >= 0) L = std::max(L, level[A[t].base]);
        }
        L += 1;
        ensure(L);
        level[w] = L;
        aff[w] = Affine{0, 1, w};
        auto &R = rows[L];
        if (nd.gate == TFHE_GATE_MUX) {
            // boot-gates.cu:407-448: u1 = woKS(-1/8 + a + b), u2 = woKS(-1/8 - a + c),
            // W = KS((0, 1/8) + u1 + u2)
            const int32_t k1[2] = {1, 1}, k2[2] = {-1, 1};
            const Affine a1[2] = {A[0], A[1]}, a2[2] = {A[0], A[2]};
            CircRow r1, r2;
            build_row(-kE8, k1, a1, 2, &r1);
            build_row(-kE8, k2, a2, 2, &r2);
            R.push_back(r1);
            R.push_back(r2);
            kss[L].push_back(CircKs{(int)R.size() - 2, (int)R.size() - 1, kE8, w});
            C->n_boot += 2;
        } else {
            CircRow r;
            build_row(nd.c0, nd.s, A, 3, &r);
            R.push_back(r);
            kss[L].push_back(CircKs{(int)R.size() - 1, -1, 0, w});
            C->n_boot += 1;
        }
    }
    C->levels.clear(); C->rows.clear(); C->ks.clear(); C->lin.clear();
    C->max_rows = 0;
    for (size_t L = 0; L < rows.size(); ++L) {
        TfheAmdCircuit::Level lv{(int)C->rows.size(), (int)rows[L].size(), (int)C->ks.size(), (int)kss[L].size(),
                                 (int)C->lin.size(), (int)lins[L].size()};
        if (lv.nrows > 65535) return TFHE_AMD_E_ARG;
        C->rows.insert(C->rows.end(), rows[L].begin(), rows[L].end());
        C->ks.insert(C->ks.end(), kss[L].begin(), kss[L].end());
        C->lin.insert(C->lin.end(), lins[L].begin(), lins[L].end());
        C->levels.push_back(lv);
        C->max_rows = std::max(C->max_rows, lv.nrows);
    }
    C->compiled = true;
    return TFHE_AMD_OK;
}

int add_node(TfheAmdCircuit *C, const Node &n) {
    const int w = (int)C->nodes.size();
    for (int t = 0; t < 3; ++t)
        if (n.in[t] < -1 || n.in[t] >= w) return TFHE_AMD_E_ARG;
    C->nodes.push_back(n);
    C->compiled = false;
    return w;
}

}  // namespace

// ------------------------------------------------------------------ C ABI

extern "C" int tfhe_amd_circuit_create(TfheAmdCircuit **out) {
    if (!out) return TFHE_AMD_E_ARG;
    *out = new TfheAmdCircuit();
    std::lock_guard<std::mutex> reg(g_circuits_mu);
    g_circuits.insert(*out);
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_circuit_destroy(TfheAmdCircuit *c) {
    if (!c) return TFHE_AMD_OK;
    {
        std::lock_guard<std::mutex> reg(g_circuits_mu);
        g_circuits.erase(c);
    }
    delete c;
    return TFHE_AMD_OK;
}

// number of contexts a circuit currently holds device state for (tests: state is dropped with
// its context)
extern "C" int tfhe_amd_circuit_state_count(TfheAmdCircuit *c) {
    if (!c) return TFHE_AMD_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    return (int)c->states.size();
}

extern "C" int tfhe_amd_circuit_inputs(TfheAmdCircuit *c, int count) {
    if (!c || count < 0) return TFHE_AMD_E_ARG;
    const int first = (int)c->nodes.size();
    for (int i = 0; i < count; ++i) c->nodes.push_back(Node{0, -1, 0, {0, 0, 0}, {-1, -1, -1}});
    c->compiled = false;
    return first;
}

extern "C" int tfhe_amd_circuit_gate(TfheAmdCircuit *c, int gate, int a, int b, int cc) {
    if (!c) return TFHE_AMD_E_ARG;
    const int ni = n_inputs(gate);
    const int in[3] = {ni > 0 ? a : -1, ni > 1 ? b : -1, ni > 2 ? cc : -1};
    for (int t = 0; t < ni; ++t)
        if (in[t] < 0) return TFHE_AMD_E_ARG;
    Node n{1, gate, 0, {0, 0, 0}, {in[0], in[1], in[2]}};
    if (gate == TFHE_GATE_NOT || gate == TFHE_GATE_COPY) n.kind = 2;
    else if (gate == TFHE_GATE_CONST) { n.kind = 2; n.c0 = a ? kE8 : -kE8; n.in[0] = -1; }
    else if (gate != TFHE_GATE_MUX && !row_spec(gate, &n.c0, &n.s[0], &n.s[1], &n.s[2])) return TFHE_AMD_E_ARG;
    return add_node(c, n);
}

extern "C" int tfhe_amd_circuit_lincomb(TfheAmdCircuit *c, int32_t c0, int32_t sa, int a, int32_t sb, int b,
                                        int32_t sc, int cc) {
    if (!c || a < 0) return TFHE_AMD_E_ARG;
    Node n{1, -1, c0, {sa, b >= 0 ? sb : 0, cc >= 0 ? sc : 0}, {a, b, cc}};
    return add_node(c, n);
}

extern "C" int tfhe_amd_circuit_node(const TfheAmdCircuit *c, int w, int *kind, int *gate, int32_t *c0, int32_t *s,
                                     int *in) {
    if (!c || w < 0 || w >= (int)c->nodes.size()) return TFHE_AMD_E_ARG;
    const Node &n = c->nodes[w];
    if (kind) *kind = n.kind;
    if (gate) *gate = n.gate;
    if (c0) *c0 = n.c0;
    for (int t = 0; t < 3; ++t) {
        if (s) s[t] = n.s[t];
        if (in) in[t] = n.in[t];
    }
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_circuit_info(TfheAmdCircuit *c, int *n_wires, int *n_gates, int *n_bootstraps,
                                     int *depth) {
    if (!c) return TFHE_AMD_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->compiled) {
        const int rc = compile(c);
        if (rc != TFHE_AMD_OK) return rc;
    }
    int ng = 0;
    for (const Node &n : c->nodes) ng += n.kind != 0;
    if (n_wires) *n_wires = (int)c->nodes.size();
    if (n_gates) *n_gates = ng;
    if (n_bootstraps) *n_bootstraps = c->n_boot;
    if (depth) *depth = (int)c->levels.size() - 1;
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_circuit_level_sizes(TfheAmdCircuit *c, int *rows_per_level, int cap) {
    if (!c) return TFHE_AMD_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->compiled) {
        const int rc = compile(c);
        if (rc != TFHE_AMD_OK) return rc;
    }
    const int nl = (int)c->levels.size();
    for (int L = 0; L < nl && L < cap; ++L) rows_per_level[L] = c->levels[L].nrows;
    return nl;
}

// wires_a [n_wires][B][500], wires_b [n_wires][B] on the context's device; input wires filled.
// The circuit's structure must not change while runs are in flight (builders invalidate the
// compiled schedule); runs on distinct contexts may overlap.
int tfhe_amd_circuit_run_dev_impl(uint64_t ctx_uid, const DeviceKey &key, int device, hipStream_t s,
                                  TfheAmdCircuit *c, int B, int32_t *wa, int32_t *wb, uint32_t *guard_stats) {
    CircuitDevState *st;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        if (!c->compiled) {
            const int rc = compile(c);
            if (rc != TFHE_AMD_OK) return rc;
            c->states.clear();   // tables of an earlier schedule
        }
        auto &slot = c->states[ctx_uid];
        if (!slot) slot.reset(new CircuitDevState());
        st = slot.get();
    }
    if (st->dev != device || !st->d_tab) {
        st->release();
        st->dev = device;
        const size_t bytes = sizeof(CircRow) * c->rows.size() + sizeof(CircKs) * c->ks.size() +
                             sizeof(CircLin) * c->lin.size() + 64;
        if (hipMalloc(&st->d_tab, bytes) != hipSuccess) return TFHE_AMD_E_NOMEM;
        char *p = (char *)st->d_tab;
        if (!c->rows.empty() && hipMemcpy(p, c->rows.data(), sizeof(CircRow) * c->rows.size(),
                                          hipMemcpyHostToDevice) != hipSuccess) return TFHE_AMD_E_HIP;
        p += sizeof(CircRow) * c->rows.size();
        if (!c->ks.empty() && hipMemcpy(p, c->ks.data(), sizeof(CircKs) * c->ks.size(),
                                        hipMemcpyHostToDevice) != hipSuccess) return TFHE_AMD_E_HIP;
        p += sizeof(CircKs) * c->ks.size();
        if (!c->lin.empty() && hipMemcpy(p, c->lin.data(), sizeof(CircLin) * c->lin.size(),
                                         hipMemcpyHostToDevice) != hipSuccess) return TFHE_AMD_E_HIP;
    }
    const size_t need = (size_t)c->max_rows * B;
    if (need > st->u_slots) {
        (void)hipDeviceSynchronize();   // the old scratch may still be in use
        if (st->u_a) (void)hipFree(st->u_a);
        if (st->u_b) (void)hipFree(st->u_b);
        if (st->u_flags) (void)hipFree(st->u_flags);
        st->u_a = nullptr; st->u_b = nullptr; st->u_flags = nullptr; st->u_slots = 0;
        if (hipMalloc(&st->u_a, sizeof(int32_t) * kN * need) != hipSuccess) return TFHE_AMD_E_NOMEM;
        if (hipMalloc(&st->u_b, sizeof(int32_t) * need) != hipSuccess) return TFHE_AMD_E_NOMEM;
        if (hipMalloc(&st->u_flags, sizeof(uint32_t) * 2 * need) != hipSuccess) return TFHE_AMD_E_NOMEM;
        st->u_slots = need;
    }
    if (st->fence.acquire(s) != hipSuccess) return TFHE_AMD_E_HIP;
    const CircRow *d_rows = (const CircRow *)st->d_tab;
    const CircKs *d_ks = (const CircKs *)(d_rows + c->rows.size());
    const CircLin *d_lin = (const CircLin *)(d_ks + c->ks.size());
    for (const auto &lv : c->levels) {
        if (lv.nrows) {
            const Guard gd = guard_stats ? Guard{st->u_flags, guard_stats} : Guard{};
            const hipError_t e =
                launch_blind_rotate_rows(key, B, lv.nrows, d_rows + lv.row0, wa, wb, kE8, st->u_a, st->u_b, s, &gd);
            if (e != hipSuccess) return TFHE_AMD_E_HIP;
            if (launch_keyswitch_rows(key, B, lv.nks, d_ks + lv.ks0, st->u_a, st->u_b, wa, wb, s) != hipSuccess)
                return TFHE_AMD_E_HIP;
        }
        if (lv.nlin && launch_circuit_linear(B, lv.nlin, d_lin + lv.lin0, wa, wb, s) != hipSuccess)
            return TFHE_AMD_E_HIP;
    }
    return st->fence.done(s) == hipSuccess ? TFHE_AMD_OK : TFHE_AMD_E_HIP;
}

// ------------------------------------------------------------------ integer builders
// Little-endian bit vectors of wire ids (bit 0 first), as Cipher.cpp stores its LweSample
// arrays.  Each builder returns a status; results are written to caller arrays.

namespace {

int G(TfheAmdCircuit *c, int gate, int a, int b = -1, int cc = -1) { return tfhe_amd_circuit_gate(c, gate, a, b, cc); }

// full adder: one level (XOR3 and MAJ side by side); cin may be -1 (zero)
void full_add(TfheAmdCircuit *c, int a, int b, int cin, int *s, int *cout) {
    if (cin < 0) {
        *s = G(c, TFHE_GATE_XOR, a, b);
        *cout = G(c, TFHE_GATE_AND, a, b);
    } else {
        *s = G(c, TFHE_GATE_XOR3, a, b, cin);
        *cout = G(c, TFHE_GATE_MAJ, a, b, cin);
    }
}

}  // namespace

// ripple-carry adder: sum[i] = a[i] ^ b[i] ^ c_i, c_{i+1} = MAJ(a[i], b[i], c_i)
// (Cipher::add / operator+, Cipher.cpp:237-276; main.cu:821-890).  Returns the carry-out wire.
extern "C" int tfhe_amd_circuit_add(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int carry_in,
                                    int *sum) {
    if (!c || nbits <= 0 || !a || !b || !sum) return TFHE_AMD_E_ARG;
    int carry = carry_in;
    for (int i = 0; i < nbits; ++i) {
        int s, co;
        full_add(c, a[i], b[i], carry, &s, &co);
        if (s < 0 || co < 0) return TFHE_AMD_E_ARG;
        sum[i] = s;
        carry = co;
    }
    return carry;
}

// a - b = a + ~b + 1 (operator-, Cipher.cpp:232-235 via twosComplement); returns the carry-out
extern "C" int tfhe_amd_circuit_sub(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int *diff) {
    if (!c || nbits <= 0 || !a || !b || !diff) return TFHE_AMD_E_ARG;
    std::vector<int> nb(nbits);
    for (int i = 0; i < nbits; ++i) nb[i] = G(c, TFHE_GATE_NOT, b[i]);
    const int one = G(c, TFHE_GATE_CONST, 1);
    return tfhe_amd_circuit_add(c, nbits, a, nb.data(), one, diff);
}

// parallel-prefix (Sklansky) adder: depth 2 + log2(nbits).  Group generate/propagate
// combine (G, P) o (G', P') = (G | (P & G'), P & P'): with G, P exclusive (p = a ^ b),
// G | (P & G') is one threshold bootstrap: 2G + P + G' - 3/8 (as +-1/8 inputs: c = +1/8).
extern "C" int tfhe_amd_circuit_add_prefix(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int *sum) {
    if (!c || nbits <= 0 || !a || !b || !sum) return TFHE_AMD_E_ARG;
    std::vector<int> g(nbits), p(nbits), G_(nbits), P_(nbits);
    for (int i = 0; i < nbits; ++i) {
        g[i] = G(c, TFHE_GATE_AND, a[i], b[i]);
        p[i] = G(c, TFHE_GATE_XOR, a[i], b[i]);
    }
    G_ = g;
    P_ = p;
    for (int d = 1; d < nbits; d <<= 1) {
        std::vector<int> Gn = G_, Pn = P_;
        for (int i = 0; i < nbits; ++i) {
            if (!(i & d)) continue;
            const int j = (i & ~(d - 1)) - 1;     // Sklansky: combine with the top of the lower block
            Gn[i] = tfhe_amd_circuit_lincomb(c, kE8, 2, G_[i], 1, P_[i], 1, G_[j]);
            Pn[i] = G(c, TFHE_GATE_AND, P_[i], P_[j]);
        }
        G_ = Gn;
        P_ = Pn;
    }
    sum[0] = p[0];
    for (int i = 1; i < nbits; ++i) sum[i] = G(c, TFHE_GATE_XOR, p[i], G_[i - 1]);
    return G_[nbits - 1];
}

namespace {

// Dadda reduction of bit columns (col[k] = wires of weight 2^k) to two rows, one level per
// stage (full adders = XOR3 + MAJ, half adders = XOR + AND; target heights 2, 3, 4, 6, 9,
// 13, ...), then a parallel-prefix adder: out[0 .. W) = the column sum mod 2^W.
void reduce_columns(TfheAmdCircuit *c, std::vector<std::vector<int>> col, int *out) {
    const int W = (int)col.size();
    size_t h0 = 0;
    for (auto &v : col) h0 = std::max(h0, v.size());
    std::vector<int> targets{2};
    while (targets.back() < (int)h0) targets.push_back(targets.back() * 3 / 2);
    for (int st = (int)targets.size() - 1; st >= 0; --st) {
        const int d = targets[st];
        size_t hmax = 0;
        for (auto &v : col) hmax = std::max(hmax, v.size());
        if ((int)hmax <= d) continue;
        std::vector<std::vector<int>> nx(W);
        for (int k = 0; k < W; ++k) {
            auto &v = col[k];
            const int cin = (int)nx[k].size();     // carries already produced into k this stage
            int h = (int)v.size();
            size_t t = 0;
            while (h + cin > d) {
                int s, co;
                if (h + cin - d >= 2 && t + 3 <= v.size()) {
                    full_add(c, v[t], v[t + 1], v[t + 2], &s, &co);
                    t += 3;
                    h -= 2;
                } else {
                    s = G(c, TFHE_GATE_XOR, v[t], v[t + 1]);
                    co = G(c, TFHE_GATE_AND, v[t], v[t + 1]);
                    t += 2;
                    h -= 1;
                }
                nx[k].push_back(s);
                if (k + 1 < W) nx[k + 1].push_back(co);
            }
            for (; t < v.size(); ++t) nx[k].push_back(v[t]);
        }
        col.swap(nx);
    }
    // two rows (missing bits = constant 0)
    int zero = -1;
    std::vector<int> x(W), y(W);
    for (int k = 0; k < W; ++k) {
        if (col[k].size() < 2 && zero < 0) zero = G(c, TFHE_GATE_CONST, 0);
        x[k] = col[k].size() > 0 ? col[k][0] : zero;
        y[k] = col[k].size() > 1 ? col[k][1] : zero;
    }
    tfhe_amd_circuit_add_prefix(c, W, x.data(), y.data(), out);
}

}  // namespace

// unsigned n x n -> 2n multiplier: n^2 partial products (one level of ANDs, the reference's
// bootsAND over iBits^2, main.cu:1506-1528), a Dadda carry-save tree and a parallel-prefix
// adder for the last two rows.  Depth 1 + stages + 2 + log2(2n).
extern "C" int tfhe_amd_circuit_mul(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int *prod) {
    if (!c || nbits <= 0 || !a || !b || !prod) return TFHE_AMD_E_ARG;
    std::vector<std::vector<int>> col(2 * nbits);
    for (int i = 0; i < nbits; ++i)
        for (int j = 0; j < nbits; ++j) col[i + j].push_back(G(c, TFHE_GATE_AND, a[j], b[i]));
    reduce_columns(c, std::move(col), prod);
    return TFHE_AMD_OK;
}

// dot product of nterms pairs of unsigned nbits integers: sum_t a_t * b_t into out_bits bits
// (mod 2^out_bits; 2 nbits + ceil(log2 nterms) bits are exact).  All nterms * nbits^2
// partial products go into ONE Dadda tree (no per-term multiplier + adder tree as in the
// reference's BOOTS_matrixMultiplication, main.cu:2342-2462): depth 1 + stages + prefix.
extern "C" int tfhe_amd_circuit_dot(TfheAmdCircuit *c, int nterms, int nbits, const int *a, const int *b,
                                    int out_bits, int *out) {
    if (!c || nterms <= 0 || nbits <= 0 || out_bits <= 0 || !a || !b || !out) return TFHE_AMD_E_ARG;
    std::vector<std::vector<int>> col(out_bits);
    for (int t = 0; t < nterms; ++t)
        for (int i = 0; i < nbits; ++i)
            for (int j = 0; j < nbits; ++j)
                if (i + j < out_bits) col[i + j].push_back(G(c, TFHE_GATE_AND, a[t * nbits + j], b[t * nbits + i]));
    reduce_columns(c, std::move(col), out);
    return TFHE_AMD_OK;
}

// ------------------------------------------------------------------ Cipher's remaining operators
// (cpuParallel/Cipher.cpp: operator> / <= / == :597-644, minimum :314-333, twosComplement
// :300-311, absolute :483-505, operator/ + divInternal + addSign :507-589), as level-batched
// circuits: each builder keeps the reference's semantics on its inputs, but replaces the
// reference's bit-serial gate chains (n dependent gates) by log-depth trees and scans.

namespace {

// Sklansky parallel-prefix carries with an optional carry-in wire (-1: none): returns the
// carry-out; sum (nullable) gets a + b + cin.  Generate / propagate as in add_prefix; the
// carry-in is the generate of a virtual bit -1 with propagate 0.
int prefix_add_cin(TfheAmdCircuit *c, int n, const int *a, const int *b, int cin, int *sum) {
    std::vector<int> g(n), p(n);
    for (int i = 0; i < n; ++i) {
        g[i] = G(c, TFHE_GATE_AND, a[i], b[i]);
        p[i] = G(c, TFHE_GATE_XOR, a[i], b[i]);
    }
    // fold the carry-in into bit 0: g0' = g0 | (p0 & cin).  g0' and p0 are no longer exclusive,
    // which the combine only needs of the upper block: a block holding bit 0 is always the lower
    std::vector<int> G_ = g, P_ = p;
    if (cin >= 0) G_[0] = tfhe_amd_circuit_lincomb(c, kE8, 2, g[0], 1, p[0], 1, cin);
    for (int d = 1; d < n; d <<= 1) {
        std::vector<int> Gn = G_, Pn = P_;
        for (int i = 0; i < n; ++i) {
            if (!(i & d)) continue;
            const int j = (i & ~(d - 1)) - 1;
            Gn[i] = tfhe_amd_circuit_lincomb(c, kE8, 2, G_[i], 1, P_[i], 1, G_[j]);
            Pn[i] = G(c, TFHE_GATE_AND, P_[i], P_[j]);
        }
        G_ = Gn;
        P_ = Pn;
    }
    if (sum) {
        sum[0] = cin >= 0 ? G(c, TFHE_GATE_XOR, p[0], cin) : p[0];
        for (int i = 1; i < n; ++i) sum[i] = G(c, TFHE_GATE_XOR, p[i], G_[i - 1]);
    }
    return G_[n - 1];
}

// carry-out of a + ~b (+ 1 if borrow_in_one): a > b (unsigned) without, a >= b with; a tree
// over the (G, P) pairs, P = XNOR (exclusive with G = a & ~b), log2 n levels
int carry_compare(TfheAmdCircuit *c, int n, const int *a, const int *b, bool ge) {
    std::vector<int> Gs(n), Ps(n);
    for (int i = 0; i < n; ++i) {
        Gs[i] = G(c, TFHE_GATE_ANDYN, a[i], b[i]);   // a & ~b
        Ps[i] = G(c, TFHE_GATE_XNOR, a[i], b[i]);    // a ^ ~b
    }
    if (ge) Gs[0] = G(c, TFHE_GATE_ORYN, a[0], b[0]);  // with carry-in 1: g0 | p0 = a0 | ~b0
    while (Gs.size() > 1) {
        std::vector<int> g2, p2;
        for (size_t i = 0; i + 1 < Gs.size(); i += 2) {   // (hi = i + 1) o (lo = i)
            g2.push_back(tfhe_amd_circuit_lincomb(c, kE8, 2, Gs[i + 1], 1, Ps[i + 1], 1, Gs[i]));
            p2.push_back(Gs.size() > 2 ? G(c, TFHE_GATE_AND, Ps[i + 1], Ps[i]) : -1);
        }
        if (Gs.size() & 1) {
            g2.push_back(Gs.back());
            p2.push_back(Ps.back());
        }
        Gs.swap(g2);
        Ps.swap(p2);
    }
    return Gs[0];
}

// prefix OR: o[i] = x[0] | ... | x[i - 1] (o[0] = none: -1), Sklansky scan
std::vector<int> prefix_or_exclusive(TfheAmdCircuit *c, int n, const int *x) {
    std::vector<int> s(x, x + n);   // inclusive scan
    for (int d = 1; d < n; d <<= 1) {
        std::vector<int> t = s;
        for (int i = 0; i < n; ++i) {
            if (!(i & d)) continue;
            const int j = (i & ~(d - 1)) - 1;
            t[i] = G(c, TFHE_GATE_OR, s[i], s[j]);
        }
        s.swap(t);
    }
    std::vector<int> o(n, -1);
    for (int i = 1; i < n; ++i) o[i] = s[i - 1];
    return o;
}

// out = cond ? -x : x (two's complement, n bits): out_i = x_i ^ (cond & (x_0 | ... | x_{i-1}))
// (cond = -1: unconditional negation, twosComplement Cipher.cpp:300-311)
void cond_negate(TfheAmdCircuit *c, int n, const int *x, int cond, int *out) {
    const std::vector<int> o = prefix_or_exclusive(c, n, x);
    out[0] = x[0];
    for (int i = 1; i < n; ++i) {
        const int t = cond >= 0 ? G(c, TFHE_GATE_AND, cond, o[i]) : o[i];
        out[i] = G(c, TFHE_GATE_XOR, x[i], t);
    }
}

}  // namespace

// comparison of two n-bit integers (two's complement when is_signed) -> one wire:
// op 0 a > b, 1 a >= b, 2 a < b, 3 a <= b, 4 a == b, 5 a != b.  operator> (Cipher.cpp:597-609)
// ripples compareBit_g = MAJ(x, ~y, c) over all bits and fixes the sign with x_msb ^ y_msb;
// here the carry of a + ~b is a log-depth (G, P) tree and the sign fix one XOR3 row.
// operator== (:628-644) ORs the bit XORs in a chain; here XNOR then an AND tree.
extern "C" int tfhe_amd_circuit_compare(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int op,
                                        int is_signed) {
    if (!c || nbits <= 0 || !a || !b || op < 0 || op > 5) return TFHE_AMD_E_ARG;
    if (op >= 4) {
        std::vector<int> e(nbits);
        for (int i = 0; i < nbits; ++i) e[i] = G(c, TFHE_GATE_XNOR, a[i], b[i]);
        while (e.size() > 1) {
            std::vector<int> e2;
            for (size_t i = 0; i + 1 < e.size(); i += 2) e2.push_back(G(c, TFHE_GATE_AND, e[i], e[i + 1]));
            if (e.size() & 1) e2.push_back(e.back());
            e.swap(e2);
        }
        return op == 4 ? e[0] : G(c, TFHE_GATE_NOT, e[0]);
    }
    // a > b = carry(a + ~b); a >= b = carry(a + ~b + 1); a < b = b > a; a <= b = b >= a
    const bool swap = op == 2 || op == 3, ge = op == 1 || op == 3;
    const int *x = swap ? b : a, *y = swap ? a : b;
    int r = carry_compare(c, nbits, x, y, ge);
    if (is_signed) r = G(c, TFHE_GATE_XOR3, r, x[nbits - 1], y[nbits - 1]);
    return r;
}

// min / max of two n-bit integers (minimum, Cipher.cpp:314-333: unsigned; is_signed: two's
// complement): one comparison, then one level of MUXes
extern "C" int tfhe_amd_circuit_minmax(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int want_max,
                                       int is_signed, int *out) {
    if (!c || nbits <= 0 || !a || !b || !out) return TFHE_AMD_E_ARG;
    const int gt = tfhe_amd_circuit_compare(c, nbits, a, b, 0, is_signed);
    if (gt < 0) return gt;
    for (int i = 0; i < nbits; ++i)
        out[i] = want_max ? G(c, TFHE_GATE_MUX, gt, a[i], b[i]) : G(c, TFHE_GATE_MUX, gt, b[i], a[i]);
    return TFHE_AMD_OK;
}

// -x (twosComplement, Cipher.cpp:300-311) and |x| (absolute, :483-505) of an n-bit two's
// complement integer: a prefix-OR scan, one AND level (abs), one XOR level
extern "C" int tfhe_amd_circuit_neg(TfheAmdCircuit *c, int nbits, const int *a, int *out) {
    if (!c || nbits <= 0 || !a || !out) return TFHE_AMD_E_ARG;
    cond_negate(c, nbits, a, -1, out);
    return TFHE_AMD_OK;
}
extern "C" int tfhe_amd_circuit_abs(TfheAmdCircuit *c, int nbits, const int *a, int *out) {
    if (!c || nbits <= 0 || !a || !out) return TFHE_AMD_E_ARG;
    cond_negate(c, nbits, a, a[nbits - 1], out);
    return TFHE_AMD_OK;
}

// unsigned restoring division q = a / b, r = a % b (n bits each; b = 0 gives q = all ones,
// r = a): for i = n - 1 .. 0: R = 2 R + a_i (n + 1 bits), T = R - b, q_i = (R >= b) = the
// carry-out of R + ~b + 1, R = q_i ? T : R.  The reference's divInternal (Cipher.cpp:526-558)
// does the same on n-bit signed intermediates; each step here is a parallel-prefix
// subtraction (depth 2 + log2(n + 1)) plus one MUX level.
extern "C" int tfhe_amd_circuit_divu(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int *q, int *r) {
    if (!c || nbits <= 0 || !a || !b || !q) return TFHE_AMD_E_ARG;
    const int n = nbits;
    const int zero = G(c, TFHE_GATE_CONST, 0), one = G(c, TFHE_GATE_CONST, 1);
    std::vector<int> R(n, zero), nb(n + 1);
    for (int i = 0; i < n; ++i) nb[i] = G(c, TFHE_GATE_NOT, b[i]);
    nb[n] = one;                                   // ~0 of the zero-extended b
    for (int i = n - 1; i >= 0; --i) {
        std::vector<int> S(n + 1);                 // 2 R + a_i
        S[0] = a[i];
        for (int k = 0; k < n; ++k) S[k + 1] = R[k];
        std::vector<int> T(n + 1);
        const int ge = prefix_add_cin(c, n + 1, S.data(), nb.data(), one, T.data());
        q[i] = ge;
        for (int k = 0; k < n; ++k) R[k] = G(c, TFHE_GATE_MUX, ge, T[k], S[k]);
    }
    if (r)
        for (int k = 0; k < n; ++k) r[k] = R[k];
    return TFHE_AMD_OK;
}

// signed division truncated toward zero (operator/, Cipher.cpp:507-524): |a| / |b| by the
// restoring divider, then negated when the signs differ (addSign :560-589)
extern "C" int tfhe_amd_circuit_div(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int *q) {
    if (!c || nbits <= 0 || !a || !b || !q) return TFHE_AMD_E_ARG;
    std::vector<int> aa(nbits), ab(nbits), uq(nbits);
    cond_negate(c, nbits, a, a[nbits - 1], aa.data());
    cond_negate(c, nbits, b, b[nbits - 1], ab.data());
    const int rc = tfhe_amd_circuit_divu(c, nbits, aa.data(), ab.data(), uq.data(), nullptr);
    if (rc < 0) return rc;
    const int sign = G(c, TFHE_GATE_XOR, a[nbits - 1], b[nbits - 1]);
    cond_negate(c, nbits, uq.data(), sign, q);
    return TFHE_AMD_OK;
}
