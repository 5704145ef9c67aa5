// Test-only CPU stand-in for the device engine (csrc/engine.cpp + the HIP kernels): the C-ABI
// entry points that the concurrency code (tfhe_api.cpp's key registry and Tier-1 coalescing
// queue, multi.cpp's multi-device registry and workers, circuit.cpp's per-context device state)
// calls, with the engine's locking discipline (one recursive mutex per context held by every
// entry point, DeviceScope around each call) and a deterministic stand-in for the gate
// arithmetic, so that tests/tsan/tsan_driver.cpp can run those modules under ThreadSanitizer
// without a GPU and compare concurrent results word for word with sequential ones.
// Not product code: the product's engine is csrc/engine.cpp.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <mutex>
#include <thread>
#include <vector>

#include "engine.h"
#include "api_internal.h"

using namespace tfhe_amd;

struct TfheAmdContext {
    int device = 0;
    hipStream_t stream = nullptr;
    bool shared_key = false;
    uint64_t uid = 0;
    std::recursive_mutex mu;
    std::vector<int32_t> last_u;   // the last batch's "extracted samples" [rows][kN]
    int last_rows = 0;
    std::vector<char> last_mux;    // mixed batches: gate i is a MUX (two rows)
};

static std::atomic<uint64_t> g_uid{1};
static std::atomic<long> g_live{0};
extern "C" long stub_live_contexts() { return g_live.load(); }
extern "C" long stub_set_device_calls() { return hip_stub::set_calls().load(); }

static void busy_wait_us(int us) {   // simulated device time: lets batches overlap
    std::this_thread::sleep_for(std::chrono::microseconds(us));
}

static bool spec(int gate, int32_t *c, int32_t *sa, int32_t *sb) {
    const int32_t e8 = 1 << 29, e4 = 1 << 30;
    switch (gate) {
    case TFHE_GATE_NAND:  *c = e8;  *sa = -1; *sb = -1; return true;
    case TFHE_GATE_OR:    *c = e8;  *sa = 1;  *sb = 1;  return true;
    case TFHE_GATE_AND:   *c = -e8; *sa = 1;  *sb = 1;  return true;
    case TFHE_GATE_XOR:   *c = e4;  *sa = 2;  *sb = 2;  return true;
    case TFHE_GATE_XNOR:  *c = -e4; *sa = -2; *sb = -2; return true;
    case TFHE_GATE_NOR:   *c = -e8; *sa = -1; *sb = -1; return true;
    case TFHE_GATE_ANDNY: *c = -e8; *sa = -1; *sb = 1;  return true;
    case TFHE_GATE_ANDYN: *c = -e8; *sa = 1;  *sb = -1; return true;
    case TFHE_GATE_ORNY:  *c = e8;  *sa = -1; *sb = 1;  return true;
    case TFHE_GATE_ORYN:  *c = e8;  *sa = 1;  *sb = -1; return true;
    default: return false;
    }
}

// stand-in "bootstrap": a deterministic mix of the row's linear combination (per coefficient)
static uint32_t mix(uint32_t x, uint32_t k) {
    x ^= k * 0x9E3779B9u;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    return x * 0xC2B2AE35u;
}
static void fake_row(int gate, const int32_t *a, int32_t ab, const int32_t *b, int32_t bb, const int32_t *c,
                     int32_t cb, int32_t *ra, int32_t *rb, int32_t *u) {
    int32_t k0, s0, s1;
    if (!spec(gate, &k0, &s0, &s1)) { k0 = 7; s0 = 3; s1 = 5; }
    for (int j = 0; j < kn; ++j) {
        uint32_t x = (uint32_t)s0 * (uint32_t)a[j] + (uint32_t)s1 * (uint32_t)b[j];
        if (c) x += 11u * (uint32_t)c[j];
        ra[j] = (int32_t)mix(x, (uint32_t)gate);
    }
    uint32_t xb = (uint32_t)k0 + (uint32_t)s0 * (uint32_t)ab + (uint32_t)s1 * (uint32_t)bb + (c ? (uint32_t)cb : 0u);
    *rb = (int32_t)mix(xb, 1u + (uint32_t)gate);
    if (u)
        for (int j = 0; j < kN; ++j) u[j] = (int32_t)mix((uint32_t)ra[j % kn] + (uint32_t)j, (uint32_t)*rb);
}

static int new_context(int device, bool shared, TfheAmdContext **out) {
    int n = 0;
    hipGetDeviceCount(&n);
    if (device < 0 || device >= n) return TFHE_AMD_E_ARG;
    TfheAmdContext *c = new TfheAmdContext();
    c->device = device;
    c->shared_key = shared;
    c->uid = g_uid++;
    DeviceScope ds(device);
    hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    g_live++;
    *out = c;
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_context_create_raw(const int32_t *bk, const int32_t *ksk, int device, TfheAmdContext **out) {
    if (!out || (!bk && !ksk)) return TFHE_AMD_E_ARG;
    busy_wait_us(300);   // key upload + conversion
    return new_context(device, false, out);
}
extern "C" int tfhe_amd_context_create_replica(TfheAmdContext *src, int device, TfheAmdContext **out) {
    if (!src || !out) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(src->mu);
    busy_wait_us(100);   // peer copies of the converted key
    return new_context(device, false, out);
}
TfheAmdContext *tfhe_amd_context_lane(TfheAmdContext *primary) {
    TfheAmdContext *c = nullptr;
    return new_context(primary->device, true, &c) == TFHE_AMD_OK ? c : nullptr;
}
extern "C" int tfhe_amd_context_destroy(TfheAmdContext *c) {
    if (!c) return TFHE_AMD_OK;
    tfhe_amd_internal_circuits_forget_context(c->uid);
    DeviceScope ds(c->device);
    {
        std::lock_guard<std::recursive_mutex> lk(c->mu);   // a batch still inside finishes first
    }
    hipStreamDestroy(c->stream);
    delete c;
    g_live--;
    return TFHE_AMD_OK;
}
extern "C" int tfhe_amd_context_device(const TfheAmdContext *c) { return c ? c->device : -1; }
extern "C" void *tfhe_amd_context_stream(TfheAmdContext *c) { return c ? (void *)c->stream : nullptr; }
extern "C" int tfhe_amd_sync(TfheAmdContext *c) { return c ? TFHE_AMD_OK : TFHE_AMD_E_ARG; }
int tfhe_amd_internal_unsliced_max() { return 1024; }

static int rows_batch(TfheAmdContext *c, int n, const int *gates, int gate, int32_t *res_a, int32_t *res_b,
                      const int32_t *a_a, const int32_t *a_b, const int32_t *b_a, const int32_t *b_b,
                      const int32_t *c_a, const int32_t *c_b) {
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope ds(c->device);
    int rows = 0;
    for (int i = 0; i < n; ++i) rows += (gates ? gates[i] : gate) == TFHE_GATE_MUX ? 2 : 1;
    // inputs are read in full before any result is written (results may alias inputs)
    std::vector<int32_t> ra((size_t)n * kn), rb(n), u((size_t)rows * kN);
    for (int i = 0, r = 0; i < n; ++i) {
        const int g = gates ? gates[i] : gate;
        const int32_t *cc = g == TFHE_GATE_MUX ? c_a + (size_t)i * kn : nullptr;
        fake_row(g, a_a + (size_t)i * kn, a_b[i], b_a + (size_t)i * kn, b_b[i], cc, cc ? c_b[i] : 0,
                 &ra[(size_t)i * kn], &rb[i], &u[(size_t)r * kN]);
        if (g == TFHE_GATE_MUX) {   // second half: u2 (the key-switch input is u1 + u2)
            for (int j = 0; j < kN; ++j) u[(size_t)(r + 1) * kN + j] = (int32_t)mix((uint32_t)j, (uint32_t)rb[i] + 5u);
            r += 2;
        } else {
            r += 1;
        }
    }
    busy_wait_us(150 + 2 * n);   // "device time" of the batch
    memcpy(res_a, ra.data(), ra.size() * 4);
    memcpy(res_b, rb.data(), rb.size() * 4);
    if (gates) {   // mixed: rows in request order
        c->last_u.swap(u);
        c->last_rows = rows;
        c->last_mux.assign(n, 0);
        for (int i = 0; i < n; ++i) c->last_mux[i] = gates[i] == TFHE_GATE_MUX;
    } else {       // gate batch: halves x B, MUX halves apart
        std::vector<int32_t> h((size_t)rows * kN);
        const int halves = gate == TFHE_GATE_MUX ? 2 : 1;
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < halves; ++k)
                memcpy(&h[((size_t)k * n + i) * kN], &u[((size_t)i * halves + k) * kN], kN * 4);
        c->last_u.swap(h);
        c->last_rows = rows;
    }
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_gate_batch_host(TfheAmdContext *c, int gate, int B, int32_t *res_a, int32_t *res_b,
                                        const int32_t *ca_a, const int32_t *ca_b, const int32_t *cb_a,
                                        const int32_t *cb_b, const int32_t *cc_a, const int32_t *cc_b) {
    int32_t k0, k1, k2;
    if (!c || B < 0 || (gate != TFHE_GATE_MUX && !spec(gate, &k0, &k1, &k2))) return TFHE_AMD_E_ARG;
    if (gate == TFHE_GATE_MUX && (!cc_a || !cc_b)) return TFHE_AMD_E_ARG;
    return rows_batch(c, B, nullptr, gate, res_a, res_b, ca_a, ca_b, cb_a, cb_b, cc_a, cc_b);
}
extern "C" int tfhe_amd_gate_batch_dev(TfheAmdContext *c, int gate, int B, int32_t *res_a, int32_t *res_b,
                                       const int32_t *ca_a, const int32_t *ca_b, const int32_t *cb_a,
                                       const int32_t *cb_b, const int32_t *cc_a, const int32_t *cc_b, void *) {
    return tfhe_amd_gate_batch_host(c, gate, B, res_a, res_b, ca_a, ca_b, cb_a, cb_b, cc_a, cc_b);
}
extern "C" int tfhe_amd_gate_batch_mixed_host(TfheAmdContext *c, int B, const int *gates, int32_t *res_a,
                                              int32_t *res_b, const int32_t *ca_a, const int32_t *ca_b,
                                              const int32_t *cb_a, const int32_t *cb_b, const int32_t *cc_a,
                                              const int32_t *cc_b) {
    if (!c || B < 0 || !gates) return TFHE_AMD_E_ARG;
    return rows_batch(c, B, gates, 0, res_a, res_b, ca_a, ca_b, cb_a, cb_b, cc_a, cc_b);
}
extern "C" int tfhe_amd_bootstrap_woks_batch_host(TfheAmdContext *c, int B, int32_t mu, const int32_t *x_a,
                                                  const int32_t *x_b, int32_t *u_a, int32_t *u_b) {
    if (!c || B < 0) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope ds(c->device);
    std::vector<int32_t> ua((size_t)B * kN), ub(B);
    for (int i = 0; i < B; ++i) {
        for (int j = 0; j < kN; ++j) ua[(size_t)i * kN + j] = (int32_t)mix((uint32_t)x_a[(size_t)i * kn + j % kn], (uint32_t)mu);
        ub[i] = (int32_t)mix((uint32_t)x_b[i], (uint32_t)mu + 1u);
    }
    busy_wait_us(100);
    memcpy(u_a, ua.data(), ua.size() * 4);
    memcpy(u_b, ub.data(), ub.size() * 4);
    return TFHE_AMD_OK;
}
extern "C" int tfhe_amd_keyswitch_batch_host(TfheAmdContext *c, int B, const int32_t *u_a, const int32_t *u_b,
                                             int32_t *res_a, int32_t *res_b) {
    if (!c || B < 0) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope ds(c->device);
    std::vector<int32_t> ra((size_t)B * kn), rb(B);
    for (int i = 0; i < B; ++i) {
        for (int j = 0; j < kn; ++j) ra[(size_t)i * kn + j] = (int32_t)mix((uint32_t)u_a[(size_t)i * kN + j], 3u);
        rb[i] = (int32_t)mix((uint32_t)u_b[i], 4u);
    }
    busy_wait_us(50);
    memcpy(res_a, ra.data(), ra.size() * 4);
    memcpy(res_b, rb.data(), rb.size() * 4);
    return TFHE_AMD_OK;
}
extern "C" int tfhe_amd_bootstrap_batch_host(TfheAmdContext *c, int B, int32_t mu, const int32_t *x_a,
                                             const int32_t *x_b, int32_t *res_a, int32_t *res_b) {
    if (!c || B < 0) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    std::vector<int32_t> ua((size_t)B * kN), ub(B);
    int rc = tfhe_amd_bootstrap_woks_batch_host(c, B, mu, x_a, x_b, ua.data(), ub.data());
    if (rc) return rc;
    c->last_u = ua;
    c->last_rows = B;
    return tfhe_amd_keyswitch_batch_host(c, B, ua.data(), ub.data(), res_a, res_b);
}
int tfhe_amd_internal_last_extracted(TfheAmdContext *c, int B, int halves, int32_t *u_a) {
    if (!c) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if ((size_t)halves * B > (size_t)c->last_rows) return TFHE_AMD_E_ARG;
    memcpy(u_a, c->last_u.data(), sizeof(int32_t) * (size_t)halves * B * kN);
    return TFHE_AMD_OK;
}
int tfhe_amd_internal_l1(TfheAmdContext *c, int op, int B, int iters, const int32_t *arg, int32_t *acc) {
    if (!c || B <= 0 || !arg || !acc) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    for (int b = 0; b < B; ++b)
        for (int j = 0; j < 2 * kN; ++j)
            acc[(size_t)b * 2 * kN + j] = (int32_t)mix((uint32_t)acc[(size_t)b * 2 * kN + j],
                                                       (uint32_t)(op == 0 ? arg[b] : iters));
    busy_wait_us(100);
    return TFHE_AMD_OK;
}
int tfhe_amd_internal_upload(TfheAmdContext *c, const void *host, size_t bytes, void **dev) {
    if (!c || !dev) return TFHE_AMD_E_ARG;
    DeviceScope ds(c->device);
    if (hipMalloc(dev, bytes) != hipSuccess) return TFHE_AMD_E_NOMEM;
    memcpy(*dev, host, bytes);
    return TFHE_AMD_OK;
}
void tfhe_amd_internal_free(int device, void *dev) {
    DeviceScope ds(device);
    hipFree(dev);
}
// the reference's order of double adds (as k_ks_variance), over the last batch's samples
int tfhe_amd_internal_ks_variance(TfheAmdContext *c, int B, int halves, const double *var, double *out) {
    if (!c) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if ((size_t)halves * B > (size_t)c->last_rows) return TFHE_AMD_E_ARG;
    for (int i = 0; i < B; ++i) {
        double v = 0.;
        for (int k = 0; k < kN; ++k) {
            uint32_t x = (uint32_t)c->last_u[(size_t)i * kN + k];
            if (halves == 2) x += (uint32_t)c->last_u[((size_t)B + i) * kN + k];
            const uint32_t aibar = x + kKsPrecOffset;
            for (int j = 0; j < kKsT; ++j) {
                const uint32_t aij = (aibar >> (32 - (j + 1) * kKsBasebit)) & (kKsBase - 1);
                if (aij) v += var[((size_t)k * kKsT + j) * kKsBase + aij];
            }
        }
        out[i] = v;
    }
    return TFHE_AMD_OK;
}
static double var_sum(const int32_t *u, const int32_t *u2, const double *var) {
    double v = 0.;
    for (int k = 0; k < kN; ++k) {
        const uint32_t aibar = (uint32_t)u[k] + (u2 ? (uint32_t)u2[k] : 0u) + kKsPrecOffset;
        for (int j = 0; j < kKsT; ++j) {
            const uint32_t aij = (aibar >> (32 - (j + 1) * kKsBasebit)) & (kKsBase - 1);
            if (aij) v += var[((size_t)k * kKsT + j) * kKsBase + aij];
        }
    }
    return v;
}
// the last mixed batch's variances (rows in request order, a MUX's two rows summed)
int tfhe_amd_internal_mixed_variance(TfheAmdContext *c, int B, const double *var, double *out) {
    if (!c || B <= 0 || !var || !out) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if ((int)c->last_mux.size() < B) return TFHE_AMD_E_ARG;
    for (int i = 0, r = 0; i < B; ++i) {
        const bool mux = c->last_mux[i];
        out[i] = var_sum(&c->last_u[(size_t)r * kN], mux ? &c->last_u[(size_t)(r + 1) * kN] : nullptr, var);
        r += mux ? 2 : 1;
    }
    return TFHE_AMD_OK;
}

// record batches (tfhe_amd_boots_batch): gather, the stand-in batch, variance, scatter, in slices
int tfhe_amd_internal_gate_batch_rows(TfheAmdContext *c, int gate, int B, const TfheAmdRows *res,
                                      const TfheAmdRows *in, int nin, const double *d_var) {
    if (!c || B < 0 || !res || !in || nin < 2 || nin > 3 || !d_var) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    auto ra_of = [](const TfheAmdRows &r, int i) {
        return *reinterpret_cast<int32_t *const *>(r.base + (size_t)i * r.stride + r.a_off);
    };
    auto rb_of = [](const TfheAmdRows &r, int i) -> int32_t & {
        return *reinterpret_cast<int32_t *>(r.base + (size_t)i * r.stride + r.b_off);
    };
    const int S = 1024, halves = gate == TFHE_GATE_MUX ? 2 : 1;
    for (int s0 = 0; s0 < B; s0 += S) {
        const int n = std::min(S, B - s0);
        std::vector<int32_t> ia((size_t)3 * n * kn), ib((size_t)3 * n), oa((size_t)n * kn), ob(n);
        for (int k = 0; k < nin; ++k)
            for (int i = 0; i < n; ++i) {
                memcpy(&ia[((size_t)k * n + i) * kn], ra_of(in[k], s0 + i), kn * 4);
                ib[(size_t)k * n + i] = rb_of(in[k], s0 + i);
            }
        const size_t na = (size_t)n * kn;
        int rc = rows_batch(c, n, nullptr, gate, oa.data(), ob.data(), ia.data(), ib.data(), ia.data() + na,
                            ib.data() + n, nin > 2 ? ia.data() + 2 * na : nullptr, nin > 2 ? ib.data() + 2 * n : nullptr);
        if (rc) return rc;
        std::vector<double> v(n);
        rc = tfhe_amd_internal_ks_variance(c, n, halves, d_var, v.data());
        if (rc) return rc;
        for (int i = 0; i < n; ++i) {
            char *rec = res->base + (size_t)(s0 + i) * res->stride;
            memcpy(*reinterpret_cast<int32_t **>(rec + res->a_off), &oa[(size_t)i * kn], kn * 4);
            *reinterpret_cast<int32_t *>(rec + res->b_off) = ob[i];
            *reinterpret_cast<double *>(rec + res->v_off) = v[i];
        }
    }
    return TFHE_AMD_OK;
}

// ---- circuits: the engine wrapper + stand-in launches (rows -> u, key switch -> wires, linear)
int tfhe_amd_circuit_run_dev_impl(uint64_t ctx_uid, const DeviceKey &key, int device, hipStream_t s,
                                  TfheAmdCircuit *c, int B, int32_t *wa, int32_t *wb, uint32_t *guard_stats);
extern "C" int tfhe_amd_circuit_run_dev(TfheAmdContext *c, TfheAmdCircuit *circ, int B, int32_t *wires_a,
                                        int32_t *wires_b, void *stream) {
    if (!c || !circ || B < 0) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope ds(c->device);
    DeviceKey key;
    key.device = c->device;
    return tfhe_amd_circuit_run_dev_impl(c->uid, key, c->device, stream ? (hipStream_t)stream : c->stream, circ, B,
                                         wires_a, wires_b, nullptr);
}
namespace tfhe_amd {
hipError_t launch_blind_rotate_rows(const DeviceKey &, int B, int nrows, const CircRow *rows, const int32_t *wa,
                                    const int32_t *wb, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t,
                                    const Guard *) {
    for (int r = 0; r < nrows; ++r)
        for (int k = 0; k < B; ++k) {
            const CircRow &w = rows[r];
            uint32_t xb = (uint32_t)w.c;
            for (int t = 0; t < 3; ++t) {
                const int wi = t == 0 ? w.x : t == 1 ? w.y : w.z;
                const int32_t s = t == 0 ? w.sa : t == 1 ? w.sb : w.sc;
                if (wi >= 0) xb += (uint32_t)s * (uint32_t)wb[(size_t)wi * B + k];
            }
            const size_t slot = (size_t)r * B + k;
            u_b[slot] = (int32_t)mix(xb, (uint32_t)mu);
            for (int j = 0; j < kN; ++j) {
                const int wi = w.x >= 0 ? w.x : 0;
                u_a[slot * kN + j] = (int32_t)mix((uint32_t)wa[((size_t)wi * B + k) * kn + j % kn] + xb, (uint32_t)j);
            }
        }
    return hipSuccess;
}
hipError_t launch_keyswitch_rows(const DeviceKey &, int B, int nks, const CircKs *ks, const int32_t *u_a,
                                 const int32_t *u_b, int32_t *wa, int32_t *wb, hipStream_t) {
    for (int o = 0; o < nks; ++o)
        for (int k = 0; k < B; ++k) {
            const CircKs &q = ks[o];
            const size_t s1 = (size_t)q.r1 * B + k;
            uint32_t b = (uint32_t)u_b[s1] + (uint32_t)q.add_b;
            if (q.r2 >= 0) b += (uint32_t)u_b[(size_t)q.r2 * B + k];
            wb[(size_t)q.out * B + k] = (int32_t)b;
            for (int j = 0; j < kn; ++j) {
                uint32_t a = (uint32_t)u_a[s1 * kN + j];
                if (q.r2 >= 0) a += (uint32_t)u_a[((size_t)q.r2 * B + k) * kN + j];
                wa[((size_t)q.out * B + k) * kn + j] = (int32_t)mix(a, 9u);
            }
        }
    return hipSuccess;
}
hipError_t launch_circuit_linear(int B, int nlin, const CircLin *lin, int32_t *wa, int32_t *wb, hipStream_t) {
    for (int o = 0; o < nlin; ++o)
        for (int k = 0; k < B; ++k) {
            const CircLin &l = lin[o];
            const size_t d = (size_t)l.out * B + k;
            uint32_t b = (uint32_t)l.c;
            if (l.in >= 0) b += (uint32_t)l.s * (uint32_t)wb[(size_t)l.in * B + k];
            wb[d] = (int32_t)b;
            for (int j = 0; j < kn; ++j)
                wa[d * kn + j] = l.in >= 0 ? (int32_t)((uint32_t)l.s * (uint32_t)wa[((size_t)l.in * B + k) * kn + j]) : 0;
        }
    return hipSuccess;
}
}  // namespace tfhe_amd
int tfhe_amd_internal_device_cus(int) { return 256; }
