// engine.cpp — device contexts, key upload, scratch and the Tier-2 (batched) C ABI.
//
// Replaces the reference GPU host glue: key upload (gpuParallel/main.cu:165-213, 236-254,
// 364-407), the per-gate chunking / temp allocation of bootsAND_fullGPU_n_Bit
// (boot-gates.cu:2845-2915) and bootstrapAndKeySwitch_n_Bit (:2481-2629).  Differences
// by design: keys are uploaded once per (cloud key, GPU) in the coefficient domain and
// converted on the device; ciphertext b-halves stay on the device; no per-call FFT plans,
// no host round trips inside a batch; work is enqueued on a caller-chosen stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <condition_variable>
#include <thread>
#include <string>
#include <vector>

#include "engine.h"
#include "api_internal.h"
#include "ntt_tables.h"
#include "../../include/tfhe_amd.h"

namespace tfhe_amd {

// ------------------------------------------------------------------ tables

uint32_t host_powmod(uint32_t b, uint64_t e, uint32_t q) {
    uint64_t r = 1, x = b % q;
    while (e) {
        if (e & 1) r = r * x % q;
        x = x * x % q;
        e >>= 1;
    }
    return (uint32_t)r;
}

static unsigned brv(unsigned x, int bits) {
    unsigned r = 0;
    for (int i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}
static uint32_t shoup(uint32_t w, uint32_t q) { return (uint32_t)(((uint64_t)w << 32) / q); }

void build_ntt_tables(NttTables *t) {
    for (int s = 0; s < 2; s++) {
        const uint32_t q = kQ[s];
        uint32_t psi = 0;
        for (uint32_t g = 2; g < 1000 && !psi; g++) {
            const uint32_t c = host_powmod(g, (q - 1) / k2N, q);
            if (host_powmod(c, kN, q) == q - 1) psi = c;   // primitive 2N-th root
        }
        const uint32_t ipsi = host_powmod(psi, q - 2, q);
        for (int k = 0; k < kN; k++) {
            t->psi[s][k] = host_powmod(psi, brv(k, kLogN), q);
            t->psip[s][k] = shoup(t->psi[s][k], q);
            t->ipsi[s][k] = host_powmod(ipsi, brv(k, kLogN), q);
            t->ipsip[s][k] = shoup(t->ipsi[s][k], q);
        }
        t->ninv[s] = host_powmod(kN, q - 2, q);
        // -q^-1 mod 2^32 by Newton iteration
        uint32_t inv = q;
        for (int it = 0; it < 5; it++) inv *= 2u - q * inv;
        t->qinv_neg[s] = 0u - inv;
        const uint32_t r_mod_q = (uint32_t)((1ull << 32) % q);
        t->bk_scale[s] = (uint32_t)((uint64_t)t->ninv[s] * r_mod_q % q);
        t->bk_scalep[s] = shoup(t->bk_scale[s], q);
    }
    t->crt_h = host_powmod(kQ[0] % kQ[1], kQ[1] - 2, kQ[1]);
    t->crt_hp = shoup(t->crt_h, kQ[1]);
}

// the calling thread's trace sink: the context of the batch entry point it is in (TraceScope)
static thread_local std::string *g_trace = nullptr;
void trace_kernel(const char *name) {
    if (!g_trace) return;
    const size_t n = strlen(name);
    for (size_t p = 0; p < g_trace->size();) {   // once per name, in first-launch order
        const size_t e = g_trace->find(',', p);
        const size_t len = (e == std::string::npos ? g_trace->size() : e) - p;
        if (len == n && g_trace->compare(p, n, name) == 0) return;
        if (e == std::string::npos) break;
        p = e + 1;
    }
    if (!g_trace->empty()) g_trace->push_back(',');
    g_trace->append(name);
}

static std::atomic<int> g_br_version{-1};

// The library carries the default fp64 kernel (v6) and the exact NTT kernel (v4: the guard's
// fallback, the L1 entry points and the exact reference generation); the earlier and experimental
// generations (v1 LDS radix-2, v2, v3, v5 latency, v7 shared-key, v8 four-wave) were retired in
// round 4 (their measurements: DESIGN.md, profiles/README.md).
static bool br_available(int v) { return v == 0 || v == 4 || v == 6; }

int br_version() {   // 0 (v6, guarded) until tfhe_amd_select_kernel picks another
    const int v = g_br_version.load(std::memory_order_relaxed);
    return v < 0 ? 0 : v;
}

// high word of the rounding distance at which the exact kernel recomputes a ciphertext: 1/8
// (0x3FC00000) by default — 1.6x the largest distance real keys show (0.06-0.08), so that an
// error can only escape by reaching 7/8 at a coefficient while every other rounding of the
// ciphertext's 500 steps stays below 1/8; tfhe_amd_set_guard_threshold lowers
// it (tests force the fallback with 0) and refuses anything above 1/8
static std::atomic<uint32_t> g_guard_hi{0x3FC00000u};
uint32_t guard_threshold_hi() { return g_guard_hi.load(std::memory_order_relaxed); }

// the default fp64 kernel, then the exact kernel in guard mode over the flags it wrote
static hipError_t run_v6_guarded(const DeviceKey &key, int B, int halves, const BrInput *in, int32_t mu,
                                 int32_t *u_a, int32_t *u_b, hipStream_t s, const Guard *guard) {
    hipError_t e = launch_blind_rotate_v6(key, B, halves, in, mu, u_a, u_b, s, guard);
    if (e != hipSuccess || !guard || !guard->flags) return e;
    return launch_blind_rotate_v4(key, B, halves, in, mu, u_a, u_b, s, guard);
}

static hipError_t run_br(const DeviceKey &key, int B, int halves, const BrInput *in, int32_t mu, int32_t *u_a,
                         int32_t *u_b, hipStream_t s, const Guard *guard) {
    switch (br_version()) {
    case 4: return launch_blind_rotate_v4(key, B, halves, in, mu, u_a, u_b, s);
    default: return run_v6_guarded(key, B, halves, in, mu, u_a, u_b, s, guard);   // 0, 6
    }
}

hipError_t launch_blind_rotate_rows(const DeviceKey &key, int B, int nrows, const CircRow *rows, const int32_t *wa,
                                    const int32_t *wb, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t s,
                                    const Guard *guard) {
    switch (br_version()) {
    case 4: return launch_blind_rotate_v4_rows(key, B, nrows, rows, wa, wb, mu, u_a, u_b, s);
    default: {
        hipError_t e = launch_blind_rotate_v6_rows(key, B, nrows, rows, wa, wb, mu, u_a, u_b, s, guard);
        if (e != hipSuccess || !guard || !guard->flags) return e;
        return launch_blind_rotate_v4_rows(key, B, nrows, rows, wa, wb, mu, u_a, u_b, s, guard);
    }
    }
}

}  // namespace tfhe_amd

using namespace tfhe_amd;

// ------------------------------------------------------------------ context

static uint64_t next_context_uid() {
    static std::atomic<uint64_t> n{1};
    return n.fetch_add(1, std::memory_order_relaxed);
}

struct TfheAmdContext {
    int device = 0;
    hipStream_t stream = nullptr;
    DeviceKey key;
    // scratch (device)
    int cap = 0;
    int32_t *u_a = nullptr;   // [2 cap][kN]   extracted samples (2 halves for MUX)
    int32_t *u_b = nullptr;   // [2 cap]
    int32_t *io = nullptr;    // host-API staging: inputs 3 x (cap x 501) + outputs cap x 501
    uint32_t *gflags = nullptr;   // exactness guard flags: 2 words per ciphertext (2 cap ciphertexts)
    uint32_t *gstats = nullptr;   // guard counters (engine.h Guard), zeroed at creation
    // pinned host staging for the host API
    int32_t *h_io = nullptr;
    void *h_u = nullptr;        // pinned readback of extracted samples (Tier-1 variance bookkeeping)
    size_t h_u_bytes = 0;
    // profiling
    bool prof = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> br_ev, ks_ev;
    double br_ms = 0, ks_ms = 0;
    int br_n = 0, ks_n = 0;
    // host-side state of the context (scratch, staging, trace string, events): every entry point
    // holds it; recursive because the host paths call the device entry points
    std::recursive_mutex mu;
    uint64_t uid = next_context_uid();   // never reused (circuit device states are keyed by it)
    bool shared_key = false;   // lane: the key belongs to another context
    StreamFence fence;         // u_a / u_b reuse across caller streams
    // sliced host batches (gate_batch_host_sliced): the input copy stream and the events
    hipStream_t copy_in = nullptr;
    hipEvent_t ev_in = nullptr, ev_out[2] = {nullptr, nullptr};
    double *d_vout = nullptr, *h_vout = nullptr;   // record batches: current_variance per result
    int vcap = 0;
    std::string last_kernels;   // kernels of the last batch entry point (tfhe_amd_last_kernels)
    void *mtab = nullptr;       // mixed-gate batches: device row / key-switch tables
    size_t mtab_bytes = 0;
    int mtab_rows = 0;          // rows of the last mixed-gate batch (its key-switch table follows them)
};

// Collects the launches of one C-ABI batch call into its context's last_kernels; nested calls
// (the host path calls the device path) keep the outermost scope's sink.
struct TraceScope {
    std::string *prev;
    explicit TraceScope(TfheAmdContext *c) : prev(g_trace) {
        if (!prev) {
            c->last_kernels.clear();
            g_trace = &c->last_kernels;
        }
    }
    ~TraceScope() {
        if (!prev) g_trace = nullptr;
    }
};

#define HIPCHK(x)                                                                 \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "tfhe_amd: %s failed: %s (%s:%d)\n", #x,              \
                    hipGetErrorString(e_), __FILE__, __LINE__);                   \
            return TFHE_AMD_E_HIP;                                                \
        }                                                                         \
    } while (0)

static int free_key(DeviceKey &k) {
    DeviceScope dev_scope(k.device);
    if (k.bk_ntt) (void)hipFree(k.bk_ntt);
    if (k.bk_v2) (void)hipFree(k.bk_v2);
    if (k.bk_fft) (void)hipFree(k.bk_fft);
    if (k.tw6) (void)hipFree(k.tw6);
    if (k.tw2) (void)hipFree(k.tw2);
    if (k.tw4) (void)hipFree(k.tw4);
    if (k.ksk) (void)hipFree(k.ksk);
    if (k.ksk4) (void)hipFree(k.ksk4);
    if (k.ksk5) (void)hipFree(k.ksk5);
    if (k.tables) (void)hipFree(k.tables);
    k = DeviceKey();
    return 0;
}

static int free_scratch(TfheAmdContext *c) {
    if (c->mtab) (void)hipFree(c->mtab);
    c->mtab = nullptr;
    c->mtab_bytes = 0;
    if (c->u_a) (void)hipFree(c->u_a);
    if (c->u_b) (void)hipFree(c->u_b);
    if (c->io) (void)hipFree(c->io);
    if (c->h_io) (void)hipHostFree(c->h_io);
    if (c->gflags) (void)hipFree(c->gflags);
    c->u_a = c->u_b = c->io = c->h_io = nullptr;
    c->gflags = nullptr;
    c->cap = 0;
    return 0;
}

static size_t io_words(int cap) { return (size_t)4 * cap * (kn + 1); }

int tfhe_amd_reserve(TfheAmdContext *c, int B) {
    if (!c || B < 0) return TFHE_AMD_E_ARG;
    if (B <= c->cap) return TFHE_AMD_OK;
    int cap = c->cap ? c->cap : 64;
    while (cap < B) cap *= 2;
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    HIPCHK(hipDeviceSynchronize());   // the scratch may still be in use on a caller's stream
    free_scratch(c);
    HIPCHK(hipMalloc(&c->u_a, sizeof(int32_t) * 2 * (size_t)cap * kN));
    HIPCHK(hipMalloc(&c->u_b, sizeof(int32_t) * 2 * (size_t)cap));
    HIPCHK(hipMalloc(&c->io, sizeof(int32_t) * io_words(cap)));
    HIPCHK(hipMalloc(&c->gflags, sizeof(uint32_t) * 4 * (size_t)cap));
    HIPCHK(hipHostMalloc(&c->h_io, sizeof(int32_t) * io_words(cap), hipHostMallocDefault));
    c->cap = cap;
    return TFHE_AMD_OK;
}

// Upload: bk [kn][4][2][kN] (nullable: KS-only context), ksk [kN][8][4][kn+1]
static int context_init(TfheAmdContext *c, const int32_t *bk, const int32_t *ksk, int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return TFHE_AMD_E_NODEVICE;
    if (device < 0 || device >= ndev) return TFHE_AMD_E_ARG;
    c->device = device;
    c->key.device = device;
    DeviceScope dev_scope(device);
    HIPCHK(dev_scope.rc);
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipMalloc(&c->gstats, sizeof(uint32_t) * 4));
    HIPCHK(hipMemset(c->gstats, 0, sizeof(uint32_t) * 4));

    NttTables *ht = new NttTables;
    build_ntt_tables(ht);
    HIPCHK(hipMalloc(&c->key.tables, sizeof(NttTables)));
    HIPCHK(hipMemcpy(c->key.tables, ht, sizeof(NttTables), hipMemcpyHostToDevice));
    c->key.qinv_neg[0] = ht->qinv_neg[0];
    c->key.qinv_neg[1] = ht->qinv_neg[1];
    c->key.crt_h = ht->crt_h;
    c->key.crt_hp = ht->crt_hp;
    {
        std::vector<uint2> tw(kTw2Words);
        build_v2_twiddles(*ht, tw.data(), tw.data() + 32, tw.data() + 64, tw.data() + 64 + 2 * 27 * 64);
        HIPCHK(hipMalloc(&c->key.tw2, sizeof(uint2) * tw.size()));
        HIPCHK(hipMemcpy(c->key.tw2, tw.data(), sizeof(uint2) * tw.size(), hipMemcpyHostToDevice));
        std::vector<uint2> tw4(kTw4Words);
        build_v4_twiddles(*ht, tw4.data(), tw4.data() + 32, tw4.data() + 32 + 2 * 27 * 64);
        HIPCHK(hipMalloc(&c->key.tw4, sizeof(uint2) * tw4.size()));
        HIPCHK(hipMemcpy(c->key.tw4, tw4.data(), sizeof(uint2) * tw4.size(), hipMemcpyHostToDevice));
        std::vector<double2> tw6(kTw6Words);
        build_v6_twiddles(tw6.data());
        HIPCHK(hipMalloc(&c->key.tw6, sizeof(double2) * tw6.size()));
        HIPCHK(hipMemcpy(c->key.tw6, tw6.data(), sizeof(double2) * tw6.size(), hipMemcpyHostToDevice));
    }
    delete ht;

    if (bk) {
        const size_t coef_words = (size_t)kn * kKpl * 2 * kN;
        int32_t *d_coef = nullptr;
        HIPCHK(hipMalloc(&d_coef, sizeof(int32_t) * coef_words));
        HIPCHK(hipMemcpy(d_coef, bk, sizeof(int32_t) * coef_words, hipMemcpyHostToDevice));
        HIPCHK(hipMalloc(&c->key.bk_ntt, sizeof(uint32_t) * 2 * coef_words));
        HIPCHK(launch_bk_to_ntt(d_coef, c->key.bk_ntt, c->key.tables, c->stream));
        HIPCHK(hipMalloc(&c->key.bk_v2, sizeof(uint32_t) * 2 * coef_words));
        HIPCHK(launch_bk_v1_to_v2(c->key.bk_ntt, c->key.bk_v2, c->stream));
        HIPCHK(hipMalloc(&c->key.bk_fft, sizeof(double2) * (size_t)kn * kKpl * 2 * 512));
        HIPCHK(launch_bk_to_fft(d_coef, c->key.bk_fft, c->key.tw6, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        HIPCHK(hipFree(d_coef));
        // the v1-layout NTT key and the NTT tables only fed the v4 repack
        HIPCHK(hipFree(c->key.bk_ntt));
        c->key.bk_ntt = nullptr;
        HIPCHK(hipFree(c->key.tables));
        c->key.tables = nullptr;
        c->key.has_bk = true;
    }
    if (ksk) {
        // drop the zero digit h = 0 (lwe-keyswitch-functions.cu:919), pad rows to 512 words
        const size_t rows = (size_t)kN * kKsT * 3;
        std::vector<int32_t> packed(rows * kKsRow, 0);
        for (int i = 0; i < kN; i++)
            for (int j = 0; j < kKsT; j++)
                for (int h = 1; h < kKsBase; h++) {
                    const int32_t *src = ksk + (((size_t)i * kKsT + j) * kKsBase + h) * (kn + 1);
                    int32_t *dst = packed.data() + (((size_t)i * kKsT + j) * 3 + (h - 1)) * kKsRow;
                    memcpy(dst, src, sizeof(int32_t) * (kn + 1));
                }
        HIPCHK(hipMalloc(&c->key.ksk, sizeof(int32_t) * packed.size()));
        HIPCHK(hipMemcpy(c->key.ksk, packed.data(), sizeof(int32_t) * packed.size(), hipMemcpyHostToDevice));
        // batches above the small-batch kernel's range: the int8 MFMA key switch (ks-v5) or,
        // with TFHE_AMD_KS5=0, ks-v4; only the chosen layout is built
        if (ks5_enabled()) {
            HIPCHK(hipMalloc(&c->key.ksk5, sizeof(int32_t) * ksk_v5_words()));
            HIPCHK(launch_ksk_to_v5(c->key.ksk, c->key.ksk5, c->stream));
        } else {
            HIPCHK(hipMalloc(&c->key.ksk4, sizeof(int32_t) * ksk_v4_words()));
            HIPCHK(launch_ksk_to_v4(c->key.ksk, c->key.ksk4, c->stream));
        }
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return tfhe_amd_reserve(c, 64);
}

extern "C" int tfhe_amd_context_create_raw(const int32_t *bk, const int32_t *ksk, int device,
                                           TfheAmdContext **out) {
    if (!out || (!bk && !ksk)) return TFHE_AMD_E_ARG;
    TfheAmdContext *c = new TfheAmdContext();
    int rc = context_init(c, bk, ksk, device);
    if (rc != TFHE_AMD_OK) {
        tfhe_amd_context_destroy(c);
        *out = nullptr;
        return rc;
    }
    *out = c;
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_context_destroy(TfheAmdContext *c) {
    if (!c) return TFHE_AMD_OK;
    tfhe_amd_internal_circuits_forget_context(c->uid);   // circuits' device state for this context
    DeviceScope dev_scope(c->device);
    (void)hipDeviceSynchronize();   // work on caller streams may still use the scratch
    for (auto &p : c->br_ev) { (void)hipEventDestroy(p.first); (void)hipEventDestroy(p.second); }
    for (auto &p : c->ks_ev) { (void)hipEventDestroy(p.first); (void)hipEventDestroy(p.second); }
    c->fence.release();
    for (hipEvent_t e : {c->ev_in, c->ev_out[0], c->ev_out[1]})
        if (e) (void)hipEventDestroy(e);
    if (c->copy_in) (void)hipStreamDestroy(c->copy_in);
    if (c->h_u) (void)hipHostFree(c->h_u);
    if (c->h_vout) (void)hipHostFree(c->h_vout);
    if (c->d_vout) (void)hipFree(c->d_vout);
    free_scratch(c);
    if (c->gstats) (void)hipFree(c->gstats);
    if (!c->shared_key) free_key(c->key);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return TFHE_AMD_OK;
}

// The device buffers of a context's key, in a fixed order: (pointer, bytes) for each domain the
// context holds (replicas, digests)
static std::vector<std::pair<void **, size_t>> key_buffers(DeviceKey &k) {
    const size_t coef = (size_t)kn * kKpl * 2 * kN;
    return {{(void **)&k.bk_ntt, k.bk_ntt ? sizeof(uint32_t) * 2 * coef : 0},
            {(void **)&k.bk_v2, k.bk_v2 ? sizeof(uint32_t) * 2 * coef : 0},
            {(void **)&k.bk_fft, k.bk_fft ? sizeof(double2) * coef / 2 : 0},
            {(void **)&k.tw2, k.tw2 ? sizeof(uint2) * kTw2Words : 0},
            {(void **)&k.tw4, k.tw4 ? sizeof(uint2) * kTw4Words : 0},
            {(void **)&k.tw6, k.tw6 ? sizeof(double2) * kTw6Words : 0},
            {(void **)&k.ksk, k.ksk ? sizeof(int32_t) * kN * kKsT * 3 * kKsRow : 0},
            {(void **)&k.ksk4, k.ksk4 ? sizeof(int32_t) * ksk_v4_words() : 0},
            {(void **)&k.ksk5, k.ksk5 ? sizeof(int32_t) * ksk_v5_words() : 0},
            {(void **)&k.tables, k.tables ? sizeof(NttTables) : 0}};
}

// A context on `device` holding a copy of src's converted device key, copied device to device
// (key replicas device 0 -> peers): hipMemcpyPeerAsync runs over xGMI when the two
// GPUs have peer access (enabled here when the driver offers it) and is staged by HIP otherwise;
// ~180 MB per key instead of the host upload + on-device conversion of every replica.
extern "C" int tfhe_amd_context_create_replica(TfheAmdContext *src, int device, TfheAmdContext **out) {
    if (!src || !out) return TFHE_AMD_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return TFHE_AMD_E_ARG;
    TfheAmdContext *c = new TfheAmdContext();
    c->device = device;
    auto fail = [&](int rc) {
        tfhe_amd_context_destroy(c);
        return rc;
    };
    DeviceScope dev_scope(device);
    if (dev_scope.rc != hipSuccess) return fail(TFHE_AMD_E_HIP);
    if (device != src->device) {
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, device, src->device) == hipSuccess && can) {
            const hipError_t e = hipDeviceEnablePeerAccess(src->device, 0);
            if (e != hipSuccess) (void)hipGetLastError();   // already enabled: fine; otherwise HIP stages
        }
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->gstats, sizeof(uint32_t) * 4) != hipSuccess ||
        hipMemset(c->gstats, 0, sizeof(uint32_t) * 4) != hipSuccess)
        return fail(TFHE_AMD_E_HIP);
    // src's lock only while its pending work (the key conversions) drains and its key is snapshot:
    // the converted key is immutable from then on, so the peer copies below run without it and the
    // replicas of several slots (multi.cpp builds them from one worker per slot) copy concurrently
    DeviceKey src_key;
    {
        std::lock_guard<std::recursive_mutex> lk(src->mu);
        DeviceScope src_scope(src->device);
        if (hipStreamSynchronize(src->stream) != hipSuccess) return fail(TFHE_AMD_E_HIP);
        src_key = src->key;
    }
    DeviceKey &k = c->key;
    k = src_key;             // scalars (CRT constants, has_bk); pointers replaced below
    k.device = device;
    auto sb = key_buffers(src_key);
    auto db = key_buffers(k);
    for (size_t i = 0; i < db.size(); ++i) *db[i].first = nullptr;
    for (size_t i = 0; i < db.size(); ++i) {
        if (!sb[i].second) continue;
        if (hipMalloc(db[i].first, sb[i].second) != hipSuccess) return fail(TFHE_AMD_E_NOMEM);
        if (hipMemcpyPeerAsync(*db[i].first, device, *sb[i].first, src->device, sb[i].second, c->stream) != hipSuccess)
            return fail(TFHE_AMD_E_HIP);
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) return fail(TFHE_AMD_E_HIP);
    const int rc = tfhe_amd_reserve(c, 64);
    if (rc != TFHE_AMD_OK) return fail(rc);
    *out = c;
    return TFHE_AMD_OK;
}

// FNV-1a 64 over the context's device key buffers (key_buffers order), read back to the host:
// tests compare a replica's bytes with its source's
extern "C" int tfhe_amd_context_key_digest(TfheAmdContext *c, unsigned long long *digest) {
    if (!c || !digest) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    HIPCHK(hipStreamSynchronize(c->stream));
    uint64_t h = 1469598103934665603ull;
    std::vector<unsigned char> buf;
    for (auto &b : key_buffers(c->key)) {
        h = (h ^ (uint64_t)b.second) * 1099511628211ull;   // which domains are present, and their sizes
        if (!b.second) continue;
        buf.resize(b.second);
        HIPCHK(hipMemcpy(buf.data(), *b.first, b.second, hipMemcpyDeviceToHost));
        for (unsigned char x : buf) h = (h ^ x) * 1099511628211ull;
    }
    *digest = h;
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_context_device(const TfheAmdContext *c) { return c ? c->device : -1; }

// device bytes held for the key material of a context (the key domains its kernels read)
extern "C" long long tfhe_amd_context_key_bytes(const TfheAmdContext *c) {
    if (!c) return TFHE_AMD_E_ARG;
    const DeviceKey &k = c->key;
    const long long bk = (long long)kn * kKpl * 2 * kN;   // coefficients per bootstrapping key
    long long n = 0;
    if (k.bk_ntt) n += bk * 2 * 4;
    if (k.bk_v2) n += bk * 2 * 4;
    if (k.bk_fft) n += bk / 2 * 16;
    if (k.tw2) n += (long long)kTw2Words * 8;
    if (k.tw4) n += (long long)kTw4Words * 8;
    if (k.tw6) n += (long long)kTw6Words * 16;
    if (k.ksk) n += (long long)kN * kKsT * 3 * kKsRow * 4;
    if (k.ksk4) n += (long long)ksk_v4_words() * 4;
    if (k.ksk5) n += (long long)ksk_v5_words() * 4;
    if (k.tables) n += (long long)sizeof(NttTables);
    return n;
}
extern "C" void *tfhe_amd_context_stream(TfheAmdContext *c) { return c ? (void *)c->stream : nullptr; }

extern "C" int tfhe_amd_sync(TfheAmdContext *c) {
    if (!c) return TFHE_AMD_E_ARG;
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    HIPCHK(hipStreamSynchronize(c->stream));
    return TFHE_AMD_OK;
}

// ------------------------------------------------------------------ profiling

static void prof_collect(TfheAmdContext *c) {
    for (auto *vec : {&c->br_ev, &c->ks_ev}) {
        for (auto &p : *vec) {
            float ms = 0;
            (void)hipEventSynchronize(p.second);
            (void)hipEventElapsedTime(&ms, p.first, p.second);
            if (vec == &c->br_ev) { c->br_ms += ms; c->br_n++; }
            else { c->ks_ms += ms; c->ks_n++; }
            (void)hipEventDestroy(p.first);
            (void)hipEventDestroy(p.second);
        }
        vec->clear();
    }
}

extern "C" int tfhe_amd_profile_enable(TfheAmdContext *c, int enable) {
    if (!c) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    prof_collect(c);
    c->prof = enable != 0;
    c->br_ms = c->ks_ms = 0;
    c->br_n = c->ks_n = 0;
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_profile_read(TfheAmdContext *c, double *br_ms, int *br_n, double *ks_ms, int *ks_n) {
    if (!c) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    prof_collect(c);
    if (br_ms) *br_ms = c->br_ms;
    if (br_n) *br_n = c->br_n;
    if (ks_ms) *ks_ms = c->ks_ms;
    if (ks_n) *ks_n = c->ks_n;
    return TFHE_AMD_OK;
}

struct ProfScope {
    TfheAmdContext *c;
    hipStream_t s;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> *vec;
    hipEvent_t a = nullptr;
    ProfScope(TfheAmdContext *c_, hipStream_t s_, bool br) : c(c_), s(s_), vec(br ? &c_->br_ev : &c_->ks_ev) {
        if (c->prof) {
            (void)hipEventCreate(&a);
            (void)hipEventRecord(a, s);
        }
    }
    ~ProfScope() {
        if (c->prof && a) {
            hipEvent_t b;
            (void)hipEventCreate(&b);
            (void)hipEventRecord(b, s);
            vec->push_back({a, b});
        }
    }
};

// ------------------------------------------------------------------ batches

static bool gate_spec(int gate, int32_t *c, int32_t *sa, int32_t *sb) {
    // constants of boot-gates.cu:98-397 (modSwitchToTorus32(+-1, 8) = +-2^29, (+-1, 4) = +-2^30)
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

static const int32_t kMu = 1 << 29;   // modSwitchToTorus32(1, 8)

// the exactness guard is always on: there is no switch that turns it off (tfhe_amd_set_guard_threshold
// can only make it stricter)
static Guard ctx_guard(TfheAmdContext *c) {
    return c->gflags && c->gstats ? Guard{c->gflags, c->gstats} : Guard{};
}

extern "C" int tfhe_amd_gate_batch_dev(TfheAmdContext *c, int gate, int B, int32_t *res_a, int32_t *res_b,
                                       const int32_t *ca_a, const int32_t *ca_b, const int32_t *cb_a,
                                       const int32_t *cb_b, const int32_t *cc_a, const int32_t *cc_b,
                                       void *stream) {
    if (!c || B < 0 || !c->key.has_bk || !c->key.ksk) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if (!res_a || !res_b || !ca_a || !ca_b || !cb_a || !cb_b) return TFHE_AMD_E_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    TraceScope trace(c);
    int rc = tfhe_amd_reserve(c, B);
    if (rc) return rc;
    HIPCHK(c->fence.acquire(s));
    if (gate == TFHE_GATE_MUX) {
        if (!cc_a || !cc_b) return TFHE_AMD_E_ARG;
        // boot-gates.cu:407-448: u1 = woKS(-1/8 + a + b), u2 = woKS(-1/8 - a + c),
        // result = KS((0, 1/8) + u1 + u2)
        BrInput in[2] = {{ca_a, ca_b, cb_a, cb_b, -kMu, 1, 1}, {ca_a, ca_b, cc_a, cc_b, -kMu, -1, 1}};
        {
            ProfScope ps(c, s, true);
            const Guard gd = ctx_guard(c);
            HIPCHK(run_br(c->key, B, 2, in, kMu, c->u_a, c->u_b, s, &gd));
        }
        ProfScope ps(c, s, false);
        HIPCHK(launch_keyswitch(c->key, B, c->u_a, c->u_b, c->u_a + (size_t)B * kN, c->u_b + B, kMu,
                                res_a, res_b, s));
        HIPCHK(c->fence.done(s));
        return TFHE_AMD_OK;
    }
    BrInput in;
    if (!gate_spec(gate, &in.c, &in.sa, &in.sb)) return TFHE_AMD_E_ARG;
    in.x_a = ca_a; in.x_b = ca_b; in.y_a = cb_a; in.y_b = cb_b;
    {
        ProfScope ps(c, s, true);
        const Guard gd = ctx_guard(c);
        HIPCHK(run_br(c->key, B, 1, &in, kMu, c->u_a, c->u_b, s, &gd));
    }
    ProfScope ps(c, s, false);
    HIPCHK(launch_keyswitch(c->key, B, c->u_a, c->u_b, nullptr, nullptr, 0, res_a, res_b, s));
    HIPCHK(c->fence.done(s));
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_bootstrap_woks_batch_dev(TfheAmdContext *c, int B, int32_t mu, const int32_t *x_a,
                                                 const int32_t *x_b, int32_t *u_a, int32_t *u_b, void *stream) {
    if (!c || B < 0 || !c->key.has_bk) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if (!x_a || !x_b || !u_a || !u_b) return TFHE_AMD_E_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    TraceScope trace(c);
    int rc = tfhe_amd_reserve(c, B);   // guard flags live in the context's scratch
    if (rc) return rc;
    HIPCHK(c->fence.acquire(s));
    BrInput in{x_a, x_b, nullptr, nullptr, 0, 1, 0};
    {
        ProfScope ps(c, s, true);
        const Guard gd = ctx_guard(c);
        HIPCHK(run_br(c->key, B, 1, &in, mu, u_a, u_b, s, &gd));
    }
    HIPCHK(c->fence.done(s));
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_bootstrap_batch_dev(TfheAmdContext *c, int B, int32_t mu, const int32_t *x_a,
                                            const int32_t *x_b, int32_t *res_a, int32_t *res_b, void *stream) {
    if (!c || B < 0 || !c->key.has_bk || !c->key.ksk) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if (!x_a || !x_b || !res_a || !res_b) return TFHE_AMD_E_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    TraceScope trace(c);
    int rc = tfhe_amd_reserve(c, B);
    if (rc) return rc;
    HIPCHK(c->fence.acquire(s));
    BrInput in{x_a, x_b, nullptr, nullptr, 0, 1, 0};
    {
        ProfScope ps(c, s, true);
        const Guard gd = ctx_guard(c);
        HIPCHK(run_br(c->key, B, 1, &in, mu, c->u_a, c->u_b, s, &gd));
    }
    ProfScope ps(c, s, false);
    HIPCHK(launch_keyswitch(c->key, B, c->u_a, c->u_b, nullptr, nullptr, 0, res_a, res_b, s));
    HIPCHK(c->fence.done(s));
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_keyswitch_batch_dev(TfheAmdContext *c, int B, const int32_t *u_a, const int32_t *u_b,
                                            int32_t *res_a, int32_t *res_b, void *stream) {
    if (!c || B < 0 || !c->key.ksk) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if (!u_a || !u_b || !res_a || !res_b) return TFHE_AMD_E_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    TraceScope trace(c);
    ProfScope ps(c, s, false);
    HIPCHK(launch_keyswitch(c->key, B, u_a, u_b, nullptr, nullptr, 0, res_a, res_b, s));
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_blind_rotate_dev(TfheAmdContext *c, int B, int iters, int32_t *acc, const int32_t *bara,
                                         void *stream) {
    if (!c || B < 0 || iters < 0 || iters > kn || !c->key.has_bk) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if (!acc || (iters > 0 && !bara)) return TFHE_AMD_E_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    TraceScope trace(c);
    ProfScope ps(c, s, true);
    const int v = br_version();
    HIPCHK(v == 4 ? launch_blind_rotate_v4_debug(c->key, B, iters, acc, bara, s)
                  : launch_blind_rotate_v6_debug(c->key, B, iters, acc, bara, s));
    return TFHE_AMD_OK;
}

// tGswFFTExternMulToTLwe (tgsw-fft-operations.cu:124-264) for B accumulators acc [B][2][kN] with
// key indices key_index [B] (device arrays): acc <- BK_i (x) acc, exact (v4 arithmetic)
extern "C" int tfhe_amd_external_product_dev(TfheAmdContext *c, int B, const int32_t *key_index, int32_t *acc,
                                             void *stream) {
    if (!c || B < 0 || !c->key.has_bk) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if (!key_index || !acc) return TFHE_AMD_E_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    TraceScope trace(c);
    HIPCHK(launch_external_product_v4(c->key, B, key_index, acc, s));
    return TFHE_AMD_OK;
}

// The L1 entry points of the TFHE API on host data (tfhe_api.cpp): op 0 = external product
// (arg = key indices [B]), op 1 = tfhe_blindRotate_FFT (arg = bara [B][iters], the exact v4 CMux
// steps, skipping a_i = 0 as lwe-bootstrapping-functions-fft.cu:705); acc [B][2][kN] in place.
int tfhe_amd_internal_l1(TfheAmdContext *c, int op, int B, int iters, const int32_t *arg, int32_t *acc) {
    if (!c || B <= 0 || !arg || !acc || !c->key.has_bk || (op == 1 && (iters < 0 || iters > kn))) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    TraceScope trace(c);
    const size_t na = op == 0 ? (size_t)B : (size_t)B * (size_t)(iters > 0 ? iters : 1);
    int32_t *d_acc = nullptr, *d_arg = nullptr;
    HIPCHK(hipMalloc(&d_acc, sizeof(int32_t) * 2 * kN * (size_t)B));
    if (hipMalloc(&d_arg, sizeof(int32_t) * na) != hipSuccess) {
        (void)hipFree(d_acc);
        return TFHE_AMD_E_NOMEM;
    }
    hipError_t e = hipMemcpyAsync(d_acc, acc, sizeof(int32_t) * 2 * kN * (size_t)B, hipMemcpyHostToDevice, c->stream);
    const size_t arg_words = op == 0 ? (size_t)B : (size_t)B * iters;
    if (e == hipSuccess && arg_words)
        e = hipMemcpyAsync(d_arg, arg, sizeof(int32_t) * arg_words, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess)
        e = op == 0 ? launch_external_product_v4(c->key, B, d_arg, d_acc, c->stream)
                    : launch_blind_rotate_v4_debug(c->key, B, iters, d_acc, d_arg, c->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(acc, d_acc, sizeof(int32_t) * 2 * kN * (size_t)B, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d_acc);
    (void)hipFree(d_arg);
    HIPCHK(e);
    return TFHE_AMD_OK;
}

// Host batches of more than one blind-rotation round are pipelined in slices of one round:
// slice s is computed on the context's stream while one copy stream moves slice s + 1 in and
// another moves slice s - 1 out, and the host stages / unstages the pinned buffers meanwhile.
// Same staging layout as below; slices touch disjoint rows, so a result that aliases an input
// (the same array) is still read before it is written.

// Host staging copies of the host-pointer paths, split over a few persistent threads: one thread
// moves ~10 GB/s, so staging a 1 024-gate batch's 4 MB of inputs and 2 MB of results took 0.17 ms
// of the call's 0.3 ms copy overhead and a 4 096-gate batch's 1 ms (scripts/host_copy_ubench.cpp,
// profiles/r04b_host_copy_ubench.jsonl: 4 threads 0.05 / 0.19 ms).  Copies below 1 MB in all, and
// calls that find the pool busy (another context copying), run on the caller's thread.
// The pool has 3 helper threads.
struct CopyJob {
    void *dst;
    const void *src;
    size_t bytes;
};
class HostCopyPool {
public:
    static HostCopyPool &get() {
        static HostCopyPool *p = new HostCopyPool();   // never destroyed: helpers idle on their cv at exit
        return *p;
    }
    void copy(const CopyJob *jobs, int n) {
        size_t total = 0;
        for (int i = 0; i < n; ++i) total += jobs[i].bytes;
        std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
        if (helpers_ == 0 || total < (1u << 20) || !busy.owns_lock()) {
            for (int i = 0; i < n; ++i) memcpy(jobs[i].dst, jobs[i].src, jobs[i].bytes);
            return;
        }
        // one immutable chunk list per job, shared with the helpers that join it (a helper still
        // finishing an earlier job holds that job's list, never this one's)
        auto job = std::make_shared<Job>();
        constexpr size_t kChunk = 256 * 1024;
        for (int i = 0; i < n; ++i)
            for (size_t o = 0; o < jobs[i].bytes; o += kChunk)
                job->chunks.push_back(CopyJob{(char *)jobs[i].dst + o, (const char *)jobs[i].src + o,
                                              std::min(kChunk, jobs[i].bytes - o)});
        job->left.store((int)job->chunks.size());
        {
            std::lock_guard<std::mutex> lk(mu_);
            cur_ = job;
            ++gen_;
        }
        cv_.notify_all();
        work(*job);
        std::unique_lock<std::mutex> lk(job->mu);
        job->done.wait(lk, [&] { return job->left.load() == 0; });
    }

private:
    struct Job {
        std::vector<CopyJob> chunks;
        std::atomic<int> next{0}, left{0};
        std::mutex mu;
        std::condition_variable done;
    };
    HostCopyPool() {
        helpers_ = 3;
        for (int i = 0; i < helpers_; ++i) std::thread([this] { loop(); }).detach();
    }
    static void work(Job &j) {
        for (;;) {
            const int i = j.next.fetch_add(1);
            if (i >= (int)j.chunks.size()) return;
            memcpy(j.chunks[i].dst, j.chunks[i].src, j.chunks[i].bytes);
            if (j.left.fetch_sub(1) == 1) {
                std::lock_guard<std::mutex> lk(j.mu);
                j.done.notify_all();
            }
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            std::shared_ptr<Job> job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                job = cur_;
            }
            if (job) work(*job);
        }
    }
    int helpers_ = 0;
    std::mutex run_mu_;                 // one copy job at a time
    std::mutex mu_;
    std::condition_variable cv_;
    uint64_t gen_ = 0;
    std::shared_ptr<Job> cur_;
};
static void host_copy(std::initializer_list<CopyJob> jobs) {
    HostCopyPool::get().copy(jobs.begin(), (int)jobs.size());
}

// TFHE_AMD_HOST_TRACE=1: one stderr line per host-pointer batch call with its host-side phases
// (ms): staging copies, waits for the device, unstaging copies, the whole call
struct HostTrace {
    static bool on() {
        static const bool v = [] {
            const char *e = getenv("TFHE_AMD_HOST_TRACE");
            return e && e[0] == '1';
        }();
        return v;
    }
    using clk = std::chrono::steady_clock;
    clk::time_point t0 = clk::now(), t = t0;
    double stage = 0, wait = 0, unstage = 0, issue = 0;
    void lap(double &acc) {
        if (!on()) return;
        const clk::time_point n = clk::now();
        acc += std::chrono::duration<double, std::milli>(n - t).count();
        t = n;
    }
    void report(const char *what, int B) {
        if (!on()) return;
        fprintf(stderr, "host_trace %s B=%d stage=%.3f issue=%.3f wait=%.3f unstage=%.3f total=%.3f\n", what, B,
                stage, issue, wait, unstage, std::chrono::duration<double, std::milli>(clk::now() - t0).count());
    }
};

// host-pointer batches above one slice are pipelined slice by slice (one unsliced batch, every
// copy in first and every copy out last, measured slower: profiles/r04o_*)
static int host_slice() { return 1024; }

static int gate_batch_host_sliced(TfheAmdContext *c, int gate, int B, int32_t *res_a, int32_t *res_b,
                                  const int32_t *const in_a[3], const int32_t *const in_b[3], int nin) {
    if (!c->copy_in) {
        HIPCHK(hipStreamCreateWithFlags(&c->copy_in, hipStreamNonBlocking));
        for (hipEvent_t *e : {&c->ev_in, &c->ev_out[0], &c->ev_out[1]})
            HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    // Staging layout (pinned h_io and device io alike): slice s's inputs as ONE contiguous block
    // at word 501 nin s0 — [a_0 | a_1 (| a_2) | b_0 | b_1 (| b_2)] — and its results at
    // 3 * 501 B + 501 s0 — [res_a | res_b].  One copy per slice and direction: the input block is
    // large enough for the copy engine (SDMA), which runs beside the blind rotation of the
    // previous slice; the small per-array copies of the round-2 layout went to blit kernels that
    // could not start while a blind rotation held every CU (rocprofv3 trace: 3.1-3.4 ms stalls),
    // serialising the pipeline.  The result copy is a blit kernel too, so it is issued on the
    // compute stream right behind its key switch, ahead of the next slice's blind rotation.
    constexpr size_t R = kn + 1;
    int32_t *h = c->h_io, *d = c->io;
    const size_t out0 = 3 * R * (size_t)B;
    const int S = host_slice();
    const int nsl = (B + S - 1) / S;
    HostTrace tr;
    auto unstage = [&](int s) -> int {
        const int s0 = s * S, n = std::min(S, B - s0);
        const int32_t *ho = h + out0 + R * (size_t)s0;
        tr.lap(tr.issue);
        HIPCHK(hipEventSynchronize(c->ev_out[s & 1]));
        tr.lap(tr.wait);
        host_copy({{res_a + (size_t)s0 * kn, ho, (size_t)n * kn * 4}, {res_b + s0, ho + (size_t)n * kn, (size_t)n * 4}});
        tr.lap(tr.unstage);
        return TFHE_AMD_OK;
    };
    for (int s = 0; s < nsl; ++s) {
        const int s0 = s * S, n = std::min(S, B - s0);
        const size_t na = (size_t)n * kn, blk = R * (size_t)nin * s0;
        int32_t *hi = h + blk, *di = d + blk;
        {
            std::vector<CopyJob> jobs;
            for (int k = 0; k < nin; ++k) {
                jobs.push_back({hi + k * na, in_a[k] + (size_t)s0 * kn, na * 4});
                jobs.push_back({hi + nin * na + (size_t)k * n, in_b[k] + s0, (size_t)n * 4});
            }
            tr.lap(tr.issue);
            HostCopyPool::get().copy(jobs.data(), (int)jobs.size());
            tr.lap(tr.stage);
        }
        HIPCHK(hipMemcpyAsync(di, hi, R * (size_t)nin * n * 4, hipMemcpyHostToDevice, c->copy_in));
        HIPCHK(hipEventRecord(c->ev_in, c->copy_in));
        HIPCHK(hipStreamWaitEvent(c->stream, c->ev_in, 0));
        const int32_t *da = di, *db = di + nin * na;
        int32_t *dout = d + out0 + R * (size_t)s0;
        const int rc = tfhe_amd_gate_batch_dev(c, gate, n, dout, dout + na, da, db, da + na, db + n,
                                               nin > 2 ? da + 2 * na : nullptr, nin > 2 ? db + 2 * n : nullptr,
                                               c->stream);
        if (rc) return rc;
        HIPCHK(hipMemcpyAsync(h + out0 + R * (size_t)s0, dout, R * (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipEventRecord(c->ev_out[s & 1], c->stream));
        if (s > 0) {
            const int r = unstage(s - 1);
            if (r) return r;
        }
    }
    const int r = unstage(nsl - 1);
    tr.report("sliced", B);
    return r;
}

// Record batches (tfhe_api.cpp tfhe_amd_boots_batch over LweSample arrays).  The records' rows
// are gathered by the copy pool straight into the pinned staging buffer (no intermediate SoA copy)
// and the results scattered back the same way; slices of one round are pipelined as in
// gate_batch_host_sliced (slice s + 1 gathered and copied in on copy_in while slice s computes,
// slice s - 1 scattered meanwhile).  Each slice's current_variance comes from k_ks_variance on the
// slice's extracted samples, queued right behind its key switch and copied out with its results.
static inline int32_t *rec_a(const TfheAmdRows &r, int i) {
    return *reinterpret_cast<int32_t *const *>(r.base + (size_t)i * r.stride + r.a_off);
}
static inline int32_t &rec_b(const TfheAmdRows &r, int i) {
    return *reinterpret_cast<int32_t *>(r.base + (size_t)i * r.stride + r.b_off);
}
static inline double &rec_v(const TfheAmdRows &r, int i) {
    return *reinterpret_cast<double *>(r.base + (size_t)i * r.stride + r.v_off);
}

int tfhe_amd_internal_gate_batch_rows(TfheAmdContext *c, int gate, int B, const TfheAmdRows *res,
                                      const TfheAmdRows *in, int nin, const double *d_var) {
    if (!c || B < 0 || !res || !in || nin < 2 || nin > 3 || !d_var) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    const bool mux = gate == TFHE_GATE_MUX;
    if (mux != (nin == 3)) return TFHE_AMD_E_ARG;
    {
        int32_t k0, k1, k2;
        if (!mux && !gate_spec(gate, &k0, &k1, &k2)) return TFHE_AMD_E_ARG;
    }
    if (!c->key.has_bk || !c->key.ksk) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    TraceScope trace(c);
    int rc = tfhe_amd_reserve(c, B);
    if (rc) return rc;
    if (!c->copy_in) {
        HIPCHK(hipStreamCreateWithFlags(&c->copy_in, hipStreamNonBlocking));
        for (hipEvent_t *e : {&c->ev_in, &c->ev_out[0], &c->ev_out[1]})
            HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    if (B > c->vcap) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->h_vout) (void)hipHostFree(c->h_vout);
        if (c->d_vout) (void)hipFree(c->d_vout);
        c->h_vout = nullptr;
        c->d_vout = nullptr;
        c->vcap = 0;
        HIPCHK(hipMalloc(&c->d_vout, sizeof(double) * (size_t)c->cap));
        HIPCHK(hipHostMalloc(&c->h_vout, sizeof(double) * (size_t)c->cap, hipHostMallocDefault));
        c->vcap = c->cap;
    }
    // staging layout as gate_batch_host_sliced: slice inputs [a_0 | a_1 (| a_2) | b_0 | b_1 (| b_2)]
    // at word R nin s0, results [res_a | res_b] at 3 R B + R s0
    constexpr size_t R = kn + 1;
    int32_t *h = c->h_io, *d = c->io;
    const size_t out0 = 3 * R * (size_t)B;
    const int S = host_slice();
    const int nsl = (B + S - 1) / S;
    const int halves = mux ? 2 : 1;
    std::vector<CopyJob> jobs;
    HostTrace tr;
    auto scatter = [&](int s) -> int {
        const int s0 = s * S, n = std::min(S, B - s0);
        const int32_t *ho = h + out0 + R * (size_t)s0;
        tr.lap(tr.issue);
        HIPCHK(hipEventSynchronize(c->ev_out[s & 1]));
        tr.lap(tr.wait);
        jobs.clear();
        for (int i = 0; i < n; ++i) jobs.push_back({rec_a(*res, s0 + i), ho + (size_t)i * kn, (size_t)kn * 4});
        HostCopyPool::get().copy(jobs.data(), (int)jobs.size());
        const int32_t *hb = ho + (size_t)n * kn;
        for (int i = 0; i < n; ++i) {
            rec_b(*res, s0 + i) = hb[i];
            rec_v(*res, s0 + i) = c->h_vout[s0 + i];
        }
        tr.lap(tr.unstage);
        return TFHE_AMD_OK;
    };
    auto drain = [&] {
        (void)hipStreamSynchronize(c->copy_in);
        (void)hipStreamSynchronize(c->stream);
    };
    for (int s = 0; s < nsl; ++s) {
        const int s0 = s * S, n = std::min(S, B - s0);
        const size_t na = (size_t)n * kn, blk = R * (size_t)nin * s0;
        int32_t *hi = h + blk, *di = d + blk;
        jobs.clear();
        for (int k = 0; k < nin; ++k)
            for (int i = 0; i < n; ++i) jobs.push_back({hi + k * na + (size_t)i * kn, rec_a(in[k], s0 + i), (size_t)kn * 4});
        tr.lap(tr.issue);
        HostCopyPool::get().copy(jobs.data(), (int)jobs.size());
        for (int k = 0; k < nin; ++k)
            for (int i = 0; i < n; ++i) hi[nin * na + (size_t)k * n + i] = rec_b(in[k], s0 + i);
        tr.lap(tr.stage);
        // one slice: the copy in on the compute stream itself (no cross-stream event on the latency path)
        hipStream_t cin = nsl > 1 ? c->copy_in : c->stream;
        hipError_t e = hipMemcpyAsync(di, hi, R * (size_t)nin * n * 4, hipMemcpyHostToDevice, cin);
        if (e == hipSuccess && nsl > 1) e = hipEventRecord(c->ev_in, c->copy_in);
        if (e == hipSuccess && nsl > 1) e = hipStreamWaitEvent(c->stream, c->ev_in, 0);
        if (e != hipSuccess) {
            drain();
            HIPCHK(e);
        }
        const int32_t *da = di, *db = di + nin * na;
        int32_t *dout = d + out0 + R * (size_t)s0;
        rc = tfhe_amd_gate_batch_dev(c, gate, n, dout, dout + na, da, db, da + na, db + n,
                                     mux ? da + 2 * na : nullptr, mux ? db + 2 * n : nullptr, c->stream);
        if (rc) {
            drain();
            return rc;
        }
        e = launch_ks_variance(c->u_a, n, halves, d_var, c->d_vout + s0, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(h + out0 + R * (size_t)s0, dout, R * (size_t)n * 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(c->h_vout + s0, c->d_vout + s0, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipEventRecord(c->ev_out[s & 1], c->stream);
        if (e != hipSuccess) {
            drain();
            HIPCHK(e);
        }
        if (s > 0 && (rc = scatter(s - 1)) != TFHE_AMD_OK) {
            drain();
            return rc;
        }
    }
    rc = scatter(nsl - 1);
    if (rc) drain();
    tr.report("records", B);
    return rc;
}

int tfhe_amd_internal_device_cus(int device) {
    static std::atomic<int> cus[64];   // per device; concurrent first calls store the same value
    const bool cached = device >= 0 && device < 64;   // an out-of-range index is queried, never cached
    int n = cached ? cus[device].load(std::memory_order_relaxed) : 0;
    if (!n) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n <= 0) {
            (void)hipGetLastError();
            n = 256;
        }
        if (cached) cus[device].store(n, std::memory_order_relaxed);
    }
    return n;
}

// Caller-owned pinned buffers.  A registry of the library's own page-locked
// allocations, [start, start + bytes): a call whose every array lies inside one of them DMAs straight
// from and to the caller's memory.  Caching hipHostRegister of arbitrary caller arrays was ruled out
// (a registration outlives a free + malloc that reuses the address); here the library
// allocates and frees, so a registered range is always the memory it was registered for.
namespace {
class PinnedRegistry {
public:
    static PinnedRegistry &get() {
        static PinnedRegistry *r = new PinnedRegistry();   // never destroyed: used from atexit paths
        return *r;
    }
    void add(void *p, size_t bytes) {
        std::lock_guard<std::mutex> lk(mu_);
        blocks_[(uintptr_t)p] = bytes;
    }
    bool remove(void *p) {
        std::lock_guard<std::mutex> lk(mu_);
        return blocks_.erase((uintptr_t)p) != 0;
    }
    bool contains(const void *p, size_t bytes) {
        if (!p) return false;
        const uintptr_t a = (uintptr_t)p;
        std::lock_guard<std::mutex> lk(mu_);
        auto it = blocks_.upper_bound(a);
        if (it == blocks_.begin()) return false;
        --it;
        return a >= it->first && bytes <= it->second && a - it->first <= it->second - bytes;
    }

private:
    std::mutex mu_;
    std::map<uintptr_t, size_t> blocks_;
};
}  // namespace

extern "C" void *tfhe_amd_host_alloc(size_t bytes) {
    if (bytes == 0) bytes = 1;
    void *p = nullptr;
    // mapped into every device's address space at the same address: the pinned path's kernels read
    // the caller's inputs through these pointers (zero-copy over PCIe), so that is checked, not assumed
    if (hipHostMalloc(&p, bytes, hipHostMallocPortable | hipHostMallocMapped) != hipSuccess || !p) {
        (void)hipGetLastError();
        return nullptr;
    }
    void *dp = nullptr;
    if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess || dp != p) {
        (void)hipGetLastError();
        (void)hipHostFree(p);
        return nullptr;
    }
    PinnedRegistry::get().add(p, bytes);
    return p;
}

extern "C" int tfhe_amd_host_free(void *p) {
    if (!p || !PinnedRegistry::get().remove(p)) return TFHE_AMD_E_ARG;
    return hipHostFree(p) == hipSuccess ? TFHE_AMD_OK : TFHE_AMD_E_HIP;
}

extern "C" int tfhe_amd_host_is_pinned(const void *p, size_t bytes) {
    return PinnedRegistry::get().contains(p, bytes) ? 1 : 0;
}

// A host batch whose arrays are all caller-owned pinned buffers: no staging and no input copy.
// Page-locked host memory is mapped into every GPU's address space, so the blind rotation's gate
// prologue (and the guard's exact recomputation) read each ciphertext's inputs straight from the
// caller's arrays over PCIe — 4 KB per ciphertext, all workgroups at once — instead of a copy in
// before the launch (r05c trace, B = 1 024: two 2 MB H2D DMAs of 41.7 us each plus two blit copies
// of the b words and the gaps between them, ~120 us before the blind rotation could start).  The
// results go the other way by DMA (the key switch writes them to device memory first: its split-K
// form adds with atomics, which are not for PCIe-mapped memory): per slice of one round, the slice's
// result copy runs on the copy stream behind its key switch while the next slice's blind rotation
// runs.  (Copying the inputs in by DMA first measured slower: 1.064x against 1.043x the device
// call at B = 1 024, profiles/r05d_*.)  Slices touch disjoint rows, so results that alias inputs are
// still read before they are written.
static int gate_batch_host_pinned(TfheAmdContext *c, int gate, int B, int32_t *res_a, int32_t *res_b,
                                  const int32_t *const in_a[3], const int32_t *const in_b[3], int nin) {
    constexpr size_t R = kn + 1;
    const int S = host_slice();
    const int nsl = (B + S - 1) / S;
    if (nsl > 1 && !c->copy_in) {
        HIPCHK(hipStreamCreateWithFlags(&c->copy_in, hipStreamNonBlocking));
        for (hipEvent_t *e : {&c->ev_in, &c->ev_out[0], &c->ev_out[1]})
            HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    int32_t *d = c->io;
    const size_t out0 = 3 * R * (size_t)B;
    HostTrace tr;
    auto drain = [&] {
        if (c->copy_in) (void)hipStreamSynchronize(c->copy_in);
        (void)hipStreamSynchronize(c->stream);
    };
    hipError_t e = hipSuccess;
    for (int s = 0; s < nsl && e == hipSuccess; ++s) {
        const int s0 = s * S, n = std::min(S, B - s0);
        const size_t na = (size_t)n * kn;
        const int32_t *xa[3], *xb[3];
        for (int k = 0; k < nin; ++k) {
            xa[k] = in_a[k] + (size_t)s0 * kn;
            xb[k] = in_b[k] + s0;
        }
        int32_t *dout = d + out0 + R * (size_t)s0;
        const int rc = tfhe_amd_gate_batch_dev(c, gate, n, dout, dout + na, xa[0], xb[0], xa[1], xb[1],
                                               nin > 2 ? xa[2] : nullptr, nin > 2 ? xb[2] : nullptr, c->stream);
        if (rc) {
            drain();
            return rc;
        }
        hipStream_t cout = c->stream;
        if (nsl > 1) {   // the result copy beside the next slice's blind rotation
            e = hipEventRecord(c->ev_out[s & 1], c->stream);
            if (e == hipSuccess) e = hipStreamWaitEvent(c->copy_in, c->ev_out[s & 1], 0);
            cout = c->copy_in;
        }
        if (e == hipSuccess) e = hipMemcpyAsync(res_a + (size_t)s0 * kn, dout, na * 4, hipMemcpyDeviceToHost, cout);
        if (e == hipSuccess) e = hipMemcpyAsync(res_b + s0, dout + na, (size_t)n * 4, hipMemcpyDeviceToHost, cout);
    }
    tr.lap(tr.issue);
    if (e == hipSuccess && nsl > 1) e = hipStreamSynchronize(c->copy_in);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    tr.lap(tr.wait);
    if (e != hipSuccess) {
        drain();
        HIPCHK(e);
    }
    tr.report("pinned", B);
    return TFHE_AMD_OK;
}

// host batch: stage inputs into pinned memory, one H2D, the device batch, one D2H (sliced and
// pipelined above one round); arrays that are all caller-owned pinned buffers skip the staging.
extern "C" int tfhe_amd_gate_batch_host(TfheAmdContext *c, int gate, int B, int32_t *res_a, int32_t *res_b,
                                        const int32_t *ca_a, const int32_t *ca_b, const int32_t *cb_a,
                                        const int32_t *cb_b, const int32_t *cc_a, const int32_t *cc_b) {
    if (!c || B < 0) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if (!res_a || !res_b || !ca_a || !ca_b || !cb_a || !cb_b) return TFHE_AMD_E_ARG;
    const bool mux = gate == TFHE_GATE_MUX;
    if (mux && (!cc_a || !cc_b)) return TFHE_AMD_E_ARG;
    {   // refuse an unknown gate before anything is staged or enqueued
        int32_t k0, k1, k2;
        if (!mux && !gate_spec(gate, &k0, &k1, &k2)) return TFHE_AMD_E_ARG;
    }
    if (!c->key.has_bk || !c->key.ksk) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    TraceScope trace(c);
    int rc = tfhe_amd_reserve(c, B);
    if (rc) return rc;
    {
        const int nin = mux ? 3 : 2;
        const int32_t *in_a[3] = {ca_a, cb_a, cc_a}, *in_b[3] = {ca_b, cb_b, cc_b};
        PinnedRegistry &pr = PinnedRegistry::get();
        const size_t A = (size_t)B * kn * 4, Bb = (size_t)B * 4;
        bool pinned = pr.contains(res_a, A) && pr.contains(res_b, Bb);
        for (int k = 0; k < nin && pinned; ++k) pinned = pr.contains(in_a[k], A) && pr.contains(in_b[k], Bb);
        if (pinned) return gate_batch_host_pinned(c, gate, B, res_a, res_b, in_a, in_b, nin);
    }
    if (B > host_slice()) {
        const int32_t *in_a[3] = {ca_a, cb_a, cc_a}, *in_b[3] = {ca_b, cb_b, cc_b};
        rc = gate_batch_host_sliced(c, gate, B, res_a, res_b, in_a, in_b, mux ? 3 : 2);
        if (rc) {
            // copies of earlier slices may still be in flight on the copy stream, not ordered
            // against the next call's staging on c->stream: drain everything before returning
            if (c->copy_in) (void)hipStreamSynchronize(c->copy_in);
            (void)hipStreamSynchronize(c->stream);
        }
        return rc;
    }
    const size_t A = (size_t)B * kn;
    // staging layout: the inputs contiguous, [ca_a | cb_a | (cc_a) | ca_b | cb_b | (cc_b)], and
    // the results [res_a | res_b] at 3 (A + B): one copy in and one copy out per call (a
    // single-gate Tier-1 call is latency-bound; each small copy is a few microseconds)
    int32_t *h = c->h_io;
    int32_t *d = c->io;
    const int nin = mux ? 3 : 2;
    const int32_t *in_a[3] = {ca_a, cb_a, cc_a}, *in_b[3] = {ca_b, cb_b, cc_b};
    int32_t *hb = h + nin * A, *db = d + nin * A;
    HostTrace tr;
    {
        // staged and copied in in two row halves above 512 gates (each >= 1 MB, so that the copy
        // pool takes it), the first half's copy in flight while the second is staged: of the copy
        // in, only the second half's stays on the call's critical path
        const int nch = B > 512 ? 2 : 1;
        std::vector<CopyJob> jobs;
        tr.lap(tr.issue);
        for (int ch = 0; ch < nch; ++ch) {
            const size_t r0 = (size_t)B * ch / nch, r1 = (size_t)B * (ch + 1) / nch;
            jobs.clear();
            for (int k = 0; k < nin; ++k) {
                jobs.push_back({h + k * A + r0 * kn, in_a[k] + r0 * kn, (r1 - r0) * kn * 4});
                jobs.push_back({hb + (size_t)k * B + r0, in_b[k] + r0, (r1 - r0) * 4});
            }
            HostCopyPool::get().copy(jobs.data(), (int)jobs.size());
            for (int k = 0; k < nin; ++k)
                HIPCHK(hipMemcpyAsync(d + k * A + r0 * kn, h + k * A + r0 * kn, (r1 - r0) * kn * 4,
                                      hipMemcpyHostToDevice, c->stream));
            if (ch == nch - 1)
                HIPCHK(hipMemcpyAsync(db, hb, (size_t)nin * B * 4, hipMemcpyHostToDevice, c->stream));
        }
        tr.lap(tr.stage);
    }
    int32_t *hr = h + 3 * (A + B), *dr = d + 3 * (A + B);
    rc = tfhe_amd_gate_batch_dev(c, gate, B, dr, dr + A, d, db, d + A, db + B,
                                 mux ? d + 2 * A : nullptr, mux ? db + 2 * B : nullptr, c->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(hr, dr, (A + B) * 4, hipMemcpyDeviceToHost, c->stream));
    tr.lap(tr.issue);
    HIPCHK(hipStreamSynchronize(c->stream));
    tr.lap(tr.wait);
    host_copy({{res_a, hr, A * 4}, {res_b, hr + A, (size_t)B * 4}});
    tr.lap(tr.unstage);
    tr.report("unsliced", B);
    return TFHE_AMD_OK;
}

// B gates of mixed kinds (gates[i] = TFHE_GATE_NAND .. TFHE_GATE_MUX) in ONE blind-rotation launch
// and ONE key-switch launch: the batch is a one-level circuit of one instance — wires 3i, 3i + 1,
// 3i + 2 hold gate i's inputs a, b (, c), wire 3B + i its result; gate i contributes one row
// (c, sa, sb) = its prologue (boot-gates.cu:98-397), a MUX two rows and a combined key switch
// (:407-448), in request order (row r of the extracted samples: gate i's first row, then its
// second for a MUX).  The rows kernel is the circuit path's k_blind_rotate_v6_rows, guarded.
// cc_* may be null when no gate is a MUX.  res may alias inputs.
extern "C" int tfhe_amd_gate_batch_mixed_host(TfheAmdContext *c, int B, const int *gates, int32_t *res_a,
                                              int32_t *res_b, const int32_t *ca_a, const int32_t *ca_b,
                                              const int32_t *cb_a, const int32_t *cb_b, const int32_t *cc_a,
                                              const int32_t *cc_b) {
    if (!c || B < 0) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if (!gates || !res_a || !res_b || !ca_a || !ca_b || !cb_a || !cb_b) return TFHE_AMD_E_ARG;
    if (!c->key.has_bk || !(c->key.ksk4 || c->key.ksk5)) return TFHE_AMD_E_ARG;
    int nmux = 0;
    for (int i = 0; i < B; ++i) {
        int32_t k0, k1, k2;
        if (gates[i] == TFHE_GATE_MUX) ++nmux;
        else if (!gate_spec(gates[i], &k0, &k1, &k2)) return TFHE_AMD_E_ARG;
    }
    if (nmux && (!cc_a || !cc_b)) return TFHE_AMD_E_ARG;
    const int rows = B + nmux;
    std::vector<CircRow> rw((size_t)rows);
    std::vector<CircKs> ks((size_t)B);
    for (int i = 0, r = 0; i < B; ++i) {
        if (gates[i] == TFHE_GATE_MUX) {
            rw[r] = CircRow{-kMu, 1, 1, 0, 3 * i, 3 * i + 1, -1, 0};
            rw[r + 1] = CircRow{-kMu, -1, 1, 0, 3 * i, 3 * i + 2, -1, 0};
            ks[i] = CircKs{r, r + 1, kMu, 3 * B + i};
            r += 2;
        } else {
            int32_t k0, k1, k2;
            gate_spec(gates[i], &k0, &k1, &k2);
            rw[r] = CircRow{k0, k1, k2, 0, 3 * i, 3 * i + 1, -1, 0};
            ks[i] = CircKs{r, -1, 0, 3 * B + i};
            r += 1;
        }
    }
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    TraceScope trace(c);
    int rc = tfhe_amd_reserve(c, std::max(B, (rows + 1) / 2));   // u / guard scratch for `rows` rows
    if (rc) return rc;
    const size_t tab = sizeof(CircRow) * rw.size() + sizeof(CircKs) * ks.size();
    if (tab > c->mtab_bytes) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->mtab) (void)hipFree(c->mtab);
        c->mtab = nullptr;
        c->mtab_bytes = 0;
        HIPCHK(hipMalloc(&c->mtab, tab));
        c->mtab_bytes = tab;
    }
    hipStream_t s = c->stream;
    HIPCHK(c->fence.acquire(s));
    // wires: a [4B][500], b [4B] in the io scratch (4 cap x 501 words), staged the same way on the host
    const size_t WA = (size_t)4 * B * kn;
    int32_t *h = c->h_io, *d = c->io;
    const int32_t *in_a[3] = {ca_a, cb_a, cc_a}, *in_b[3] = {ca_b, cb_b, cc_b};
    for (int i = 0; i < B; ++i)
        for (int k = 0; k < (gates[i] == TFHE_GATE_MUX ? 3 : 2); ++k) {
            memcpy(h + (size_t)(3 * i + k) * kn, in_a[k] + (size_t)i * kn, kn * 4);
            h[WA + 3 * i + k] = in_b[k][i];
        }
    HIPCHK(hipMemcpyAsync(d, h, (size_t)3 * B * kn * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d + WA, h + WA, (size_t)3 * B * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->mtab, rw.data(), sizeof(CircRow) * rw.size(), hipMemcpyHostToDevice, s));
    const CircKs *d_ks = (const CircKs *)((char *)c->mtab + sizeof(CircRow) * rw.size());
    c->mtab_rows = rows;
    HIPCHK(hipMemcpyAsync((void *)d_ks, ks.data(), sizeof(CircKs) * ks.size(), hipMemcpyHostToDevice, s));
    {
        ProfScope ps(c, s, true);
        const Guard gd = ctx_guard(c);
        HIPCHK(launch_blind_rotate_rows(c->key, 1, rows, (const CircRow *)c->mtab, d, d + WA, kMu, c->u_a, c->u_b, s,
                                        &gd));
    }
    {
        ProfScope ps(c, s, false);
        HIPCHK(launch_keyswitch_rows(c->key, 1, B, d_ks, c->u_a, c->u_b, d, d + WA, s));
    }
    int32_t *hr = h + (size_t)3 * B * kn;
    HIPCHK(hipMemcpyAsync(hr, d + (size_t)3 * B * kn, (size_t)B * kn * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(h + WA + 3 * B, d + WA + 3 * B, (size_t)B * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c->fence.done(s));
    HIPCHK(hipStreamSynchronize(s));   // also: the host tables above may be freed on return
    memcpy(res_a, hr, (size_t)B * kn * 4);
    memcpy(res_b, h + WA + 3 * B, (size_t)B * 4);
    return TFHE_AMD_OK;
}

// woKS / bootstrap / KS host versions: same staging scheme (in-place safe)
enum { OP_WOKS, OP_BOOT, OP_KS };
static int single_input_host(TfheAmdContext *c, int op, int B, int32_t mu, const int32_t *in_a,
                             const int32_t *in_b, int32_t *out_a, int32_t *out_b) {
    if (!c || B < 0) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if (!in_a || !in_b || !out_a || !out_b) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    TraceScope trace(c);
    int rc = tfhe_amd_reserve(c, B);
    if (rc) return rc;
    const int din = op == OP_KS ? kN : kn, dout = op == OP_WOKS ? kN : kn;
    const size_t Ai = (size_t)B * din, Ao = (size_t)B * dout;
    int32_t *h = c->h_io, *d = c->io;
    // [in_a | in_b | out_a | out_b]  (<= B * (1025 + 1025) words <= 4 * cap * 501)
    memcpy(h, in_a, Ai * 4);
    memcpy(h + Ai, in_b, (size_t)B * 4);
    HIPCHK(hipMemcpyAsync(d, h, (Ai + B) * 4, hipMemcpyHostToDevice, c->stream));
    int32_t *oa = d + Ai + B, *ob = oa + Ao;
    if (op == OP_WOKS) rc = tfhe_amd_bootstrap_woks_batch_dev(c, B, mu, d, d + Ai, oa, ob, c->stream);
    else if (op == OP_BOOT) rc = tfhe_amd_bootstrap_batch_dev(c, B, mu, d, d + Ai, oa, ob, c->stream);
    else rc = tfhe_amd_keyswitch_batch_dev(c, B, d, d + Ai, oa, ob, c->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(h + Ai + B, oa, (Ao + B) * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(out_a, h + Ai + B, Ao * 4);
    memcpy(out_b, h + Ai + B + Ao, (size_t)B * 4);
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_bootstrap_woks_batch_host(TfheAmdContext *c, int B, int32_t mu, const int32_t *x_a,
                                                  const int32_t *x_b, int32_t *u_a, int32_t *u_b) {
    return single_input_host(c, OP_WOKS, B, mu, x_a, x_b, u_a, u_b);
}
extern "C" int tfhe_amd_bootstrap_batch_host(TfheAmdContext *c, int B, int32_t mu, const int32_t *x_a,
                                             const int32_t *x_b, int32_t *res_a, int32_t *res_b) {
    return single_input_host(c, OP_BOOT, B, mu, x_a, x_b, res_a, res_b);
}
extern "C" int tfhe_amd_keyswitch_batch_host(TfheAmdContext *c, int B, const int32_t *u_a, const int32_t *u_b,
                                             int32_t *res_a, int32_t *res_b) {
    return single_input_host(c, OP_KS, B, 0, u_a, u_b, res_a, res_b);
}

// largest batch the host path runs unsliced, i.e. whose key-switch inputs are all in the scratch
// afterwards (tfhe_api.cpp's variance bookkeeping rounds)
int tfhe_amd_internal_unsliced_max() { return host_slice(); }

// The extracted samples (key-switch inputs) of this context's last gate batch of at most one
// round (unsliced host path), halves x B rows of kN words: the Tier-1 API's per-thread-lane mode
// (TFHE_AMD_TIER1_COALESCE=0) and raw tfhe_bootstrap_FFT derive the key-switched output's
// current_variance from their digits (tfhe_api.cpp ks_variance).
int tfhe_amd_internal_last_extracted(TfheAmdContext *c, int B, int halves, int32_t *u_a) {
    if (!c || B <= 0 || halves < 1 || halves > 2 || (size_t)halves * B > 2 * (size_t)c->cap) return TFHE_AMD_E_ARG;
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    const size_t bytes = sizeof(int32_t) * (size_t)halves * B * kN;
    // through the context's pinned readback buffer: a D2H straight into the caller's (pageable,
    // often freshly allocated) array costs a fixed ~0.3 ms per call
    if (bytes > c->h_u_bytes) {
        if (c->h_u) (void)hipHostFree(c->h_u);
        c->h_u = nullptr;
        c->h_u_bytes = 0;
        HIPCHK(hipHostMalloc(&c->h_u, bytes, hipHostMallocDefault));
        c->h_u_bytes = bytes;
    }
    HIPCHK(hipMemcpyAsync(c->h_u, c->u_a, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    host_copy({{u_a, c->h_u, bytes}});
    return TFHE_AMD_OK;
}

// device copy of host data on a context's GPU (tfhe_api.cpp: the KSK row variances)
int tfhe_amd_internal_upload(TfheAmdContext *c, const void *host, size_t bytes, void **dev) {
    if (!c || !host || !dev) return TFHE_AMD_E_ARG;
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    HIPCHK(hipMalloc(dev, bytes));
    HIPCHK(hipMemcpy(*dev, host, bytes, hipMemcpyHostToDevice));
    return TFHE_AMD_OK;
}
void tfhe_amd_internal_free(int device, void *dev) {
    if (!dev) return;
    DeviceScope dev_scope(device);
    (void)hipFree(dev);
}

// current_variance of the context's last gate batch (<= one round: its key-switch inputs are still
// in the scratch), computed on the device (k_ks_variance) into out [B]
int tfhe_amd_internal_ks_variance(TfheAmdContext *c, int B, int halves, const double *d_var, double *out) {
    if (!c || B <= 0 || halves < 1 || halves > 2 || (size_t)halves * B > 2 * (size_t)c->cap || !d_var || !out)
        return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    double *d_out = reinterpret_cast<double *>(c->io);   // the batch's staging is done with by now
    HIPCHK(launch_ks_variance(c->u_a, B, halves, d_var, d_out, c->stream));
    HIPCHK(hipMemcpyAsync(out, d_out, sizeof(double) * (size_t)B, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return TFHE_AMD_OK;
}

// current_variance of the context's last mixed-gate batch (tfhe_amd_gate_batch_mixed_host: its row and
// key-switch tables and extracted samples are still in the scratch), on the device, into out [B]
int tfhe_amd_internal_mixed_variance(TfheAmdContext *c, int B, const double *d_var, double *out) {
    if (!c || B <= 0 || !d_var || !out || !c->mtab || c->mtab_rows < B) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    if (B > c->vcap) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->h_vout) (void)hipHostFree(c->h_vout);
        if (c->d_vout) (void)hipFree(c->d_vout);
        c->h_vout = nullptr;
        c->d_vout = nullptr;
        c->vcap = 0;
        HIPCHK(hipMalloc(&c->d_vout, sizeof(double) * (size_t)c->cap));
        HIPCHK(hipHostMalloc(&c->h_vout, sizeof(double) * (size_t)c->cap, hipHostMallocDefault));
        c->vcap = c->cap;
    }
    const CircKs *d_ks = (const CircKs *)((char *)c->mtab + sizeof(CircRow) * (size_t)c->mtab_rows);
    HIPCHK(launch_ks_variance_rows(c->u_a, B, d_ks, d_var, c->d_vout, c->stream));
    HIPCHK(hipMemcpyAsync(c->h_vout, c->d_vout, sizeof(double) * (size_t)B, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(out, c->h_vout, sizeof(double) * (size_t)B);
    return TFHE_AMD_OK;
}

// a second context on the same GPU sharing `primary`'s key (own stream + scratch):
// used for per-thread lanes of the Tier-1 API
TfheAmdContext *tfhe_amd_context_lane(TfheAmdContext *primary) {
    TfheAmdContext *c = new TfheAmdContext();
    c->device = primary->device;
    c->key = primary->key;
    c->shared_key = true;
    DeviceScope dev_scope(c->device);
    if (dev_scope.rc != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->gstats, sizeof(uint32_t) * 4) != hipSuccess ||
        hipMemset(c->gstats, 0, sizeof(uint32_t) * 4) != hipSuccess ||
        tfhe_amd_reserve(c, 64) != TFHE_AMD_OK) {
        tfhe_amd_context_destroy(c);
        return nullptr;
    }
    return c;
}

// circuit.cpp
int tfhe_amd_circuit_run_dev_impl(uint64_t ctx_uid, const DeviceKey &key, int device, hipStream_t s,
                                  TfheAmdCircuit *c, int B, int32_t *wa, int32_t *wb, uint32_t *guard_stats);

extern "C" int tfhe_amd_circuit_run_dev(TfheAmdContext *c, TfheAmdCircuit *circ, int B, int32_t *wires_a,
                                        int32_t *wires_b, void *stream) {
    if (!c || !circ || B < 0 || !c->key.has_bk || !(c->key.ksk4 || c->key.ksk5)) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if (!wires_a || !wires_b) return TFHE_AMD_E_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    TraceScope trace(c);
    return tfhe_amd_circuit_run_dev_impl(c->uid, c->key, c->device, s, circ, B, wires_a, wires_b, c->gstats);
}

extern "C" int tfhe_amd_set_guard_threshold(double distance) {
    // stricter than the default only: a threshold above 1/8 would let a rounding error of up to
    // 1 - threshold escape
    if (!(distance >= 0.0 && distance <= 0.125)) return TFHE_AMD_E_ARG;
    uint64_t bits;
    memcpy(&bits, &distance, 8);
    g_guard_hi.store((uint32_t)(bits >> 32));
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_guard_stats(TfheAmdContext *c, double *max_distance, long long *recomputed, int reset) {
    if (!c || !c->gstats) return TFHE_AMD_E_ARG;
    DeviceScope dev_scope(c->device);
    HIPCHK(dev_scope.rc);
    HIPCHK(hipDeviceSynchronize());   // launches on caller streams update the counters
    uint32_t h[4];
    HIPCHK(hipMemcpy(h, c->gstats, sizeof h, hipMemcpyDeviceToHost));
    if (max_distance) {
        const uint64_t bits = (uint64_t)h[1] << 32;   // high word: the distance rounded down
        double d;
        memcpy(&d, &bits, 8);
        *max_distance = d;
    }
    if (recomputed) *recomputed = h[0];
    if (reset) HIPCHK(hipMemset(c->gstats, 0, sizeof h));
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_last_kernels(TfheAmdContext *c, char *buf, int cap) {
    if (!c || !buf || cap <= 0) return TFHE_AMD_E_ARG;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    const size_t n = std::min(c->last_kernels.size(), (size_t)cap - 1);
    memcpy(buf, c->last_kernels.data(), n);
    buf[n] = 0;
    return (int)c->last_kernels.size();
}

extern "C" int tfhe_amd_select_kernel(int br_version) {
    if (!br_available(br_version)) return TFHE_AMD_E_ARG;
    g_br_version.store(br_version);
    return TFHE_AMD_OK;
}

extern "C" const char *tfhe_amd_version(void) {
    // one immutable string per (blind-rotation, key-switch) generation pair
    static char names[8][6][48];
    static std::once_flag once;
    std::call_once(once, [] {
        for (int b = 0; b <= 7; b++)
            for (int k = 1; k <= 5; k++) {
                if (b == 0 || b >= 6)
                    snprintf(names[b][k], sizeof names[b][k], "tfhe_amd gfx950 fft64 br-v%d ks-v%d", 6, k);
                else snprintf(names[b][k], sizeof names[b][k], "tfhe_amd gfx950 ntt2x27 br-v%d ks-v%d", b, k);
            }
    });
    return names[br_version()][ks_version()];
}
