// multi.cpp — one process driving several GPUs (SURVEY.md §8(e), §8(b) Tier-2 tfhe_gpu_init /
// tfhe_gpu_boots_batch).
//
// The reference runs its GPU gate batches on one device and walks a batch in chunks
// (bootsAND_fullGPU_n_Bit, gpuParallel/boot-gates.cu:2869-2907).  Here a batch of independent
// gates is split into contiguous per-device shards (sizes differ by at most one, the same
// arithmetic as shard.py's shard_range), every device holds a full replica of the key (its own
// TfheAmdContext: FFT- and NTT-domain bootstrapping keys + key-switching layouts, uploaded once),
// and one persistent worker thread per device stages its shard, runs it (the single-device host
// path: pinned staging, a copy stream, one-round launches) and copies it back.  There is no
// collective: the shards are independent and land in disjoint rows of the caller's arrays.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "params.h"
#include "../../include/tfhe/tfhe.h"
#include "../../include/tfhe_amd.h"
#include "api_internal.h"

using namespace tfhe_amd;

// contiguous shard [lo, hi) of `total` independent gates for `rank` of `world` (shard.py)
extern "C" int tfhe_amd_shard_range(long long total, int rank, int world, long long *lo, long long *hi) {
    if (world <= 0 || rank < 0 || rank >= world || total < 0 || !lo || !hi) return TFHE_AMD_E_ARG;
    const long long per = total / world, extra = total % world;
    *lo = rank * per + (rank < extra ? rank : extra);
    *hi = *lo + per + (rank < extra ? 1 : 0);
    return TFHE_AMD_OK;
}

namespace {

// one worker thread per device: runs one job at a time, the caller waits for all of them
class Worker {
public:
    Worker() : th_([this] { loop(); }) {}
    ~Worker() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    void submit(std::function<int()> job) {
        std::lock_guard<std::mutex> lk(mu_);
        job_ = std::move(job);
        done_ = false;
        cv_.notify_all();
    }
    int wait() {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return done_; });
        return rc_;
    }

private:
    void loop() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [this] { return stop_ || (job_ && !done_); });
            if (stop_) return;
            std::function<int()> job = std::move(job_);
            job_ = nullptr;
            lk.unlock();
            const int rc = job();
            lk.lock();
            rc_ = rc;
            done_ = true;
            cv_.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::function<int()> job_;
    bool done_ = true, stop_ = false;
    int rc_ = 0;
    std::thread th_;   // last: starts after the members above exist
};

}  // namespace

struct TfheAmdMulti {
    std::vector<int> devices;
    std::vector<TfheAmdContext *> ctx;
    std::vector<std::unique_ptr<Worker>> workers;
    std::mutex mu;   // one batch at a time per multi-context
};

extern "C" int tfhe_amd_multi_destroy(TfheAmdMulti *m) {
    if (!m) return TFHE_AMD_OK;
    { std::lock_guard<std::mutex> lk(m->mu); }   // a batch still running on it finishes first
    m->workers.clear();   // joins the threads
    for (auto *c : m->ctx)
        if (c) tfhe_amd_context_destroy(c);
    delete m;
    return TFHE_AMD_OK;
}

// bk int32 [500][4][2][1024], ksk int32 [1024][8][4][501]; devices may repeat (several
// contexts on one GPU: the split path on a single-GPU machine)
extern "C" int tfhe_amd_multi_create_raw(const int32_t *bk, const int32_t *ksk, const int *devices, int ndev,
                                         TfheAmdMulti **out) {
    if (!bk || !ksk || !devices || ndev <= 0 || !out) return TFHE_AMD_E_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return TFHE_AMD_E_NODEVICE;
    for (int i = 0; i < ndev; ++i)
        if (devices[i] < 0 || devices[i] >= count) return TFHE_AMD_E_ARG;
    TfheAmdMulti *m = new TfheAmdMulti();
    m->devices.assign(devices, devices + ndev);
    m->ctx.assign(ndev, nullptr);
    for (int i = 0; i < ndev; ++i) m->workers.emplace_back(new Worker());
    // slot 0's key is uploaded and converted on its device; the other slots copy slot 0's converted
    // key device to device (peer copies over xGMI, concurrently, one worker per slot: SURVEY.md §5).
    int rc = tfhe_amd_context_create_raw(bk, ksk, m->devices[0], &m->ctx[0]);
    for (int i = 1; i < ndev && rc == TFHE_AMD_OK; ++i)
        m->workers[i]->submit([=] { return tfhe_amd_context_create_replica(m->ctx[0], m->devices[i], &m->ctx[i]); });
    for (int i = 1; i < ndev && m->ctx[0]; ++i) {
        const int r = m->workers[i]->wait();
        if (r != TFHE_AMD_OK && rc == TFHE_AMD_OK) rc = r;
    }
    if (rc != TFHE_AMD_OK) {
        tfhe_amd_multi_destroy(m);
        return rc;
    }
    *out = m;
    return TFHE_AMD_OK;
}

extern "C" int tfhe_amd_multi_create(const TFheGateBootstrappingCloudKeySet *bk, int device_mask, TfheAmdMulti **out) {
    if (!bk || !bk->bkFFT || !out || device_mask <= 0) return TFHE_AMD_E_ARG;
    std::vector<int> devs;
    for (int d = 0; d < 31; ++d)
        if (device_mask & (1 << d)) devs.push_back(d);
    if (devs.empty()) return TFHE_AMD_E_ARG;
    std::vector<int32_t> flat_bk((size_t)kn * kKpl * 2 * kN), flat_ks((size_t)kN * kKsT * kKsBase * (kn + 1));
    if (tfhe_amd_internal_bk_coef(bk, flat_bk.data()) != TFHE_AMD_OK || tfhe_amd_export_ksk(bk, flat_ks.data()) != TFHE_AMD_OK)
        return TFHE_AMD_E_ARG;
    return tfhe_amd_multi_create_raw(flat_bk.data(), flat_ks.data(), devs.data(), (int)devs.size(), out);
}

extern "C" int tfhe_amd_multi_devices(const TfheAmdMulti *m, int *devices, int cap) {
    if (!m) return TFHE_AMD_E_ARG;
    for (int i = 0; i < (int)m->devices.size() && i < cap; ++i) devices[i] = m->devices[i];
    return (int)m->devices.size();
}

extern "C" TfheAmdContext *tfhe_amd_multi_context(TfheAmdMulti *m, int i) {
    return m && i >= 0 && i < (int)m->ctx.size() ? m->ctx[i] : nullptr;
}

// B gates split over the devices; host arrays (SoA), synchronous; res may alias inputs (every
// shard reads its rows before writing them, and shards are disjoint)
extern "C" int tfhe_amd_multi_gate_batch_host(TfheAmdMulti *m, int gate, int B, int32_t *res_a, int32_t *res_b,
                                              const int32_t *ca_a, const int32_t *ca_b, const int32_t *cb_a,
                                              const int32_t *cb_b, const int32_t *cc_a, const int32_t *cc_b) {
    if (!m || B < 0) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if (!res_a || !res_b || !ca_a || !ca_b || !cb_a || !cb_b) return TFHE_AMD_E_ARG;
    if (gate == TFHE_GATE_MUX && (!cc_a || !cc_b)) return TFHE_AMD_E_ARG;
    if (gate < TFHE_GATE_NAND || gate > TFHE_GATE_MUX) return TFHE_AMD_E_ARG;
    std::lock_guard<std::mutex> lk(m->mu);
    const int world = (int)m->ctx.size();
    int used = 0;
    for (int r = 0; r < world; ++r) {
        long long lo, hi;
        tfhe_amd_shard_range(B, r, world, &lo, &hi);
        if (hi == lo) continue;
        const size_t o = (size_t)lo * kn;
        const int n = (int)(hi - lo);
        TfheAmdContext *c = m->ctx[r];
        m->workers[r]->submit([=] {
            return tfhe_amd_gate_batch_host(c, gate, n, res_a + o, res_b + lo, ca_a + o, ca_b + lo, cb_a + o,
                                            cb_b + lo, cc_a ? cc_a + o : nullptr, cc_b ? cc_b + lo : nullptr);
        });
        used = r + 1;
    }
    int rc = TFHE_AMD_OK;
    for (int r = 0; r < used; ++r) {
        long long lo, hi;
        tfhe_amd_shard_range(B, r, world, &lo, &hi);
        if (hi == lo) continue;
        const int x = m->workers[r]->wait();
        if (x != TFHE_AMD_OK && rc == TFHE_AMD_OK) rc = x;
    }
    return rc;
}

// Device-resident shards: slot i's shard (counts[i] gates) already lives on that slot's device;
// the batch is enqueued on every slot (streams[i], or the slot context's own stream when streams or
// streams[i] is NULL) and the call returns without waiting (tfhe_amd_multi_sync).  No PCIe in the
// loop: the shards' inputs and results stay in each device's HBM.
extern "C" int tfhe_amd_multi_gate_batch_dev(TfheAmdMulti *m, int gate, const int *counts, int32_t *const *res_a,
                                             int32_t *const *res_b, const int32_t *const *ca_a,
                                             const int32_t *const *ca_b, const int32_t *const *cb_a,
                                             const int32_t *const *cb_b, const int32_t *const *cc_a,
                                             const int32_t *const *cc_b, void *const *streams) {
    if (!m || !counts || !res_a || !res_b || !ca_a || !ca_b || !cb_a || !cb_b) return TFHE_AMD_E_ARG;
    if (gate < TFHE_GATE_NAND || gate > TFHE_GATE_MUX) return TFHE_AMD_E_ARG;
    if (gate == TFHE_GATE_MUX && (!cc_a || !cc_b)) return TFHE_AMD_E_ARG;
    const int world = (int)m->ctx.size();
    for (int r = 0; r < world; ++r)
        if (counts[r] < 0) return TFHE_AMD_E_ARG;
    std::lock_guard<std::mutex> lk(m->mu);
    for (int r = 0; r < world; ++r) {
        if (counts[r] == 0) continue;
        const int rc = tfhe_amd_gate_batch_dev(m->ctx[r], gate, counts[r], res_a[r], res_b[r], ca_a[r], ca_b[r],
                                               cb_a[r], cb_b[r], cc_a ? cc_a[r] : nullptr, cc_b ? cc_b[r] : nullptr,
                                               streams ? streams[r] : nullptr);
        if (rc != TFHE_AMD_OK) return rc;
    }
    return TFHE_AMD_OK;
}

// waits for every slot context's own stream
extern "C" int tfhe_amd_multi_sync(TfheAmdMulti *m) {
    if (!m) return TFHE_AMD_E_ARG;
    int rc = TFHE_AMD_OK;
    for (auto *c : m->ctx) {
        const int x = tfhe_amd_sync(c);
        if (x != TFHE_AMD_OK && rc == TFHE_AMD_OK) rc = x;
    }
    return rc;
}

// A circuit over the devices, device-resident: slot i evaluates counts[i] instances in its own
// wire arrays wires_a[i] [n_wires][counts[i]][500], wires_b[i] [n_wires][counts[i]] (input wires
// filled).  Enqueued on every slot, returns without waiting.
extern "C" int tfhe_amd_multi_circuit_run_dev(TfheAmdMulti *m, TfheAmdCircuit *circ, const int *counts,
                                              int32_t *const *wires_a, int32_t *const *wires_b,
                                              void *const *streams) {
    if (!m || !circ || !counts || !wires_a || !wires_b) return TFHE_AMD_E_ARG;
    const int world = (int)m->ctx.size();
    for (int r = 0; r < world; ++r)
        if (counts[r] < 0 || (counts[r] > 0 && (!wires_a[r] || !wires_b[r]))) return TFHE_AMD_E_ARG;
    int rc = tfhe_amd_circuit_info(circ, nullptr, nullptr, nullptr, nullptr);   // compile once, here
    if (rc != TFHE_AMD_OK) return rc;
    std::lock_guard<std::mutex> lk(m->mu);
    for (int r = 0; r < world; ++r) {
        if (counts[r] == 0) continue;
        rc = tfhe_amd_circuit_run_dev(m->ctx[r], circ, counts[r], wires_a[r], wires_b[r],
                                      streams ? streams[r] : nullptr);
        if (rc != TFHE_AMD_OK) return rc;
    }
    return TFHE_AMD_OK;
}

namespace {

// copies `nw` wires between the caller's host planes [nw][B][ld] (instance rows lo..lo+n) and a
// device wire array [n_wires][n][ld], one 2-D copy per run of consecutive wire ids
int copy_planes(int32_t *dev, const int *wires, int nw, int32_t *host, long long B, long long lo, int n, int ld,
                bool to_device, hipStream_t s) {
    for (int k0 = 0; k0 < nw;) {
        int k1 = k0 + 1;
        while (k1 < nw && wires[k1] == wires[k1 - 1] + 1) ++k1;
        int32_t *d = dev + (size_t)wires[k0] * n * ld;
        int32_t *h = host + ((size_t)k0 * B + lo) * ld;
        const size_t dp = (size_t)n * ld * 4, hp = (size_t)B * ld * 4;
        const hipError_t e = to_device ? hipMemcpy2DAsync(d, dp, h, hp, dp, k1 - k0, hipMemcpyHostToDevice, s)
                                       : hipMemcpy2DAsync(h, hp, d, dp, dp, k1 - k0, hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) return TFHE_AMD_E_HIP;
        k0 = k1;
    }
    return TFHE_AMD_OK;
}

}  // namespace

// A circuit over the devices from host memory: B instances split into contiguous shards (as
// tfhe_amd_shard_range); every device copies in its shard of the n_in input wires
// (in_a [n_in][B][500], in_b [n_in][B]: plane k is wire in_wires[k]), evaluates the circuit in its
// own HBM wire arrays and copies back its shard of the n_out wires out_wires into out_a
// [n_out][B][500], out_b [n_out][B].  Synchronous.  Generalizes the reference's matrix-vector
// product over a device (BOOTS_matrixMultiplication, gpuParallel/main.cu:2342-2462; row layout
// matrixUtility.cu:65-96) to all of a node's GPUs from one host process.
extern "C" int tfhe_amd_multi_circuit_run_host(TfheAmdMulti *m, TfheAmdCircuit *circ, int B, int n_in,
                                               const int *in_wires, const int32_t *in_a, const int32_t *in_b,
                                               int n_out, const int *out_wires, int32_t *out_a, int32_t *out_b) {
    if (!m || !circ || B < 0 || n_in < 0 || n_out < 0) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if ((n_in && (!in_wires || !in_a || !in_b)) || (n_out && (!out_wires || !out_a || !out_b))) return TFHE_AMD_E_ARG;
    int n_wires = 0;
    int rc = tfhe_amd_circuit_info(circ, &n_wires, nullptr, nullptr, nullptr);   // compile once, here
    if (rc != TFHE_AMD_OK) return rc;
    for (int k = 0; k < n_in; ++k)
        if (in_wires[k] < 0 || in_wires[k] >= n_wires) return TFHE_AMD_E_ARG;
    for (int k = 0; k < n_out; ++k)
        if (out_wires[k] < 0 || out_wires[k] >= n_wires) return TFHE_AMD_E_ARG;
    std::lock_guard<std::mutex> lk(m->mu);
    const int world = (int)m->ctx.size();
    std::vector<int> used;
    for (int r = 0; r < world; ++r) {
        long long lo, hi;
        tfhe_amd_shard_range(B, r, world, &lo, &hi);
        if (hi == lo) continue;
        const int n = (int)(hi - lo);
        TfheAmdContext *c = m->ctx[r];
        const int dev = m->devices[r];
        m->workers[r]->submit([=]() -> int {
            if (hipSetDevice(dev) != hipSuccess) return TFHE_AMD_E_HIP;
            hipStream_t s = (hipStream_t)tfhe_amd_context_stream(c);
            int32_t *wa = nullptr, *wb = nullptr;
            if (hipMalloc(&wa, sizeof(int32_t) * (size_t)n_wires * n * kn) != hipSuccess) return TFHE_AMD_E_NOMEM;
            if (hipMalloc(&wb, sizeof(int32_t) * (size_t)n_wires * n) != hipSuccess) {
                (void)hipFree(wa);
                return TFHE_AMD_E_NOMEM;
            }
            int x = copy_planes(wa, in_wires, n_in, const_cast<int32_t *>(in_a), B, lo, n, kn, true, s);
            if (!x) x = copy_planes(wb, in_wires, n_in, const_cast<int32_t *>(in_b), B, lo, n, 1, true, s);
            if (!x) x = tfhe_amd_circuit_run_dev(c, circ, n, wa, wb, s);
            if (!x) x = copy_planes(wa, out_wires, n_out, out_a, B, lo, n, kn, false, s);
            if (!x) x = copy_planes(wb, out_wires, n_out, out_b, B, lo, n, 1, false, s);
            if (hipStreamSynchronize(s) != hipSuccess && !x) x = TFHE_AMD_E_HIP;
            (void)hipFree(wa);
            (void)hipFree(wb);
            return x;
        });
        used.push_back(r);
    }
    for (int r : used) {
        const int x = m->workers[r]->wait();
        if (x != TFHE_AMD_OK && rc == TFHE_AMD_OK) rc = x;
    }
    return rc;
}

// ------------------------------------------------------------------ SURVEY.md §8(b) Tier-2 names
// tfhe_gpu_init registers a multi-device context for a cloud key; tfhe_gpu_boots_batch runs a
// batch of one gate over it (falling back to the key's Tier-1 device when not registered).

// Registered multi-contexts are shared: a batch holds its own reference for the whole call, so a
// concurrent tfhe_gpu_init (re-registration) or key deletion only drops the registry's reference
// and the last in-flight batch frees the contexts and joins the workers.
static std::mutex g_multi_mu;
static std::unordered_map<const void *, std::shared_ptr<TfheAmdMulti>> g_multi;   // bkFFT -> multi-context

static std::shared_ptr<TfheAmdMulti> share_multi(TfheAmdMulti *m) {
    return std::shared_ptr<TfheAmdMulti>(m, [](TfheAmdMulti *p) { tfhe_amd_multi_destroy(p); });
}

extern "C" int tfhe_gpu_init(const TFheGateBootstrappingCloudKeySet *bk, int device_mask) {
    if (!bk || !bk->bkFFT) return TFHE_AMD_E_ARG;
    TfheAmdMulti *m = nullptr;
    const int rc = tfhe_amd_multi_create(bk, device_mask, &m);
    if (rc != TFHE_AMD_OK) return rc;
    std::shared_ptr<TfheAmdMulti> old;   // released outside the registry lock (may join workers)
    {
        std::lock_guard<std::mutex> lk(g_multi_mu);
        auto it = g_multi.find(bk->bkFFT);
        if (it != g_multi.end()) old = std::move(it->second);
        g_multi[bk->bkFFT] = share_multi(m);
    }
    return TFHE_AMD_OK;
}

// drop the multi-context of a key being deleted (tfhe_api.cpp delete_* hooks)
void tfhe_amd_internal_forget_multi(const void *bkfft) {
    std::shared_ptr<TfheAmdMulti> m;   // in-flight batches keep their own reference
    {
        std::lock_guard<std::mutex> lk(g_multi_mu);
        auto it = g_multi.find(bkfft);
        if (it == g_multi.end()) return;
        m = std::move(it->second);
        g_multi.erase(it);
    }
}

extern "C" int tfhe_gpu_boots_batch(int gate, int32_t *res_a, int32_t *res_b, const int32_t *a_a, const int32_t *a_b,
                                    const int32_t *b_a, const int32_t *b_b, const int32_t *c_a, const int32_t *c_b,
                                    int B, const TFheGateBootstrappingCloudKeySet *bk) {
    if (!bk || !bk->bkFFT) return TFHE_AMD_E_ARG;
    std::shared_ptr<TfheAmdMulti> m;   // held for the whole batch (see g_multi)
    {
        std::lock_guard<std::mutex> lk(g_multi_mu);
        auto it = g_multi.find(bk->bkFFT);
        if (it != g_multi.end()) m = it->second;
    }
    if (m) return tfhe_amd_multi_gate_batch_host(m.get(), gate, B, res_a, res_b, a_a, a_b, b_a, b_b, c_a, c_b);
    return tfhe_amd_internal_tier1_batch(bk, gate, B, res_a, res_b, a_a, a_b, b_a, b_b, c_a, c_b);
}
