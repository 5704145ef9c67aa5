// ThreadSanitizer driver for the device engine's host side (VERDICT r4 item 4;
// tests/test_concurrency_tsan.py): csrc/engine.cpp itself — its host copy pool (HostCopyPool,
// shared by every context), the pinned-buffer registry, the staged / sliced / record / pinned host
// paths, the context lock, key replicas — built unchanged with -fsanitize=thread against the
// asynchronous stub HIP runtime (stub/hip/hip_runtime.h: streams are worker threads) and CPU
// stand-in kernels (stub_kernels.cpp), together with the rest of the host library.
//
// Phases (every concurrent result is compared word for word, current_variance bit for bit, with
// the same work run sequentially on one context first):
//   1. host batches from T threads over three contexts (two devices, one a replica built while
//      the others run): staged (one round, two halves through the copy pool), sliced (1 100 and a
//      2 100-gate MUX: slices of 1 024 pipelined over the copy stream), caller-owned pinned arrays,
//      and record batches (LweSample-like rows: gather into pinned staging, scatter back,
//      current_variance on the device) — several threads on ONE context at once;
//   2. the pinned registry under churn: host_alloc / host_free from some threads while others
//      query is_pinned and run pinned batches.
// Exit 0 = all equal; ThreadSanitizer itself exits 66 on any report.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "engine.h"
#include "api_internal.h"
#include "../../include/tfhe_amd.h"

static std::atomic<int> g_fail{0};
#define CHECK(cond, ...)                                         \
    do {                                                         \
        if (!(cond)) {                                           \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                        \
            fprintf(stderr, "\n");                               \
            g_fail = 1;                                          \
        }                                                        \
    } while (0)

using tfhe_amd::kn;

static uint32_t lcg(uint32_t &s) { return s = s * 1664525u + 1013904223u; }

enum Path { STAGED = 0, PINNED = 1, RECORDS = 2 };
static const char *kPath[] = {"staged", "pinned", "records"};

struct Rec {   // an LweSample-like record: pointer to a[500], b, current_variance
    int32_t *a;
    int32_t b;
    double var;
};

struct Work {
    int gate, B, path;
    uint32_t seed;
    std::vector<int32_t> in_a[3], in_b[3];   // the inputs (nin of them)
    std::vector<int32_t> want_a, want_b;     // sequential results
    std::vector<double> want_v;              // records: current_variance
    int nin() const { return gate == TFHE_GATE_MUX ? 3 : 2; }
};

static void make_inputs(Work &w) {
    uint32_t s = w.seed;
    for (int k = 0; k < w.nin(); ++k) {
        w.in_a[k].resize((size_t)w.B * kn);
        w.in_b[k].resize(w.B);
        for (auto &x : w.in_a[k]) x = (int32_t)lcg(s);
        for (auto &x : w.in_b[k]) x = (int32_t)lcg(s);
    }
}

// one run of a workload on a context; results (and variances) returned
static int run(TfheAmdContext *c, const Work &w, const double *d_var, std::vector<int32_t> &ra,
               std::vector<int32_t> &rb, std::vector<double> &rv) {
    const int B = w.B, nin = w.nin();
    ra.assign((size_t)B * kn, 0);
    rb.assign(B, 0);
    rv.clear();
    if (w.path == STAGED) {
        return tfhe_amd_gate_batch_host(c, w.gate, B, ra.data(), rb.data(), w.in_a[0].data(), w.in_b[0].data(),
                                        w.in_a[1].data(), w.in_b[1].data(), nin > 2 ? w.in_a[2].data() : nullptr,
                                        nin > 2 ? w.in_b[2].data() : nullptr);
    }
    if (w.path == PINNED) {
        const size_t A = (size_t)B * kn * 4, Bb = (size_t)B * 4;
        int32_t *pa[4], *pb[4];
        for (int k = 0; k < 4; ++k) {
            pa[k] = (int32_t *)tfhe_amd_host_alloc(A);
            pb[k] = (int32_t *)tfhe_amd_host_alloc(Bb);
            if (!pa[k] || !pb[k]) return -4;
        }
        for (int k = 0; k < nin; ++k) {
            memcpy(pa[k], w.in_a[k].data(), A);
            memcpy(pb[k], w.in_b[k].data(), Bb);
        }
        CHECK(tfhe_amd_host_is_pinned(pa[0] + 7, 64) == 1 && tfhe_amd_host_is_pinned(pa[0], A + 4) == 0,
              "registry bounds");
        const int rc = tfhe_amd_gate_batch_host(c, w.gate, B, pa[3], pb[3], pa[0], pb[0], pa[1], pb[1],
                                                nin > 2 ? pa[2] : nullptr, nin > 2 ? pb[2] : nullptr);
        memcpy(ra.data(), pa[3], A);
        memcpy(rb.data(), pb[3], Bb);
        for (int k = 0; k < 4; ++k) {
            CHECK(tfhe_amd_host_free(pa[k]) == 0 && tfhe_amd_host_free(pb[k]) == 0, "host_free");
        }
        return rc;
    }
    // records: inputs and results as arrays of LweSample-like records, results written into the
    // first input's records (in place, as Cipher.cpp:387's callers do)
    std::vector<std::vector<int32_t>> store((size_t)nin * B, std::vector<int32_t>(kn));
    std::vector<Rec> recs((size_t)nin * B);
    for (int k = 0; k < nin; ++k)
        for (int i = 0; i < B; ++i) {
            Rec &r = recs[(size_t)k * B + i];
            r.a = store[(size_t)k * B + i].data();
            memcpy(r.a, &w.in_a[k][(size_t)i * kn], kn * 4);
            r.b = w.in_b[k][i];
            r.var = -1.0;
        }
    TfheAmdRows in[3], res;
    for (int k = 0; k < nin; ++k)
        in[k] = TfheAmdRows{(char *)&recs[(size_t)k * B], sizeof(Rec), offsetof(Rec, a), offsetof(Rec, b),
                            offsetof(Rec, var)};
    res = in[0];
    const int rc = tfhe_amd_internal_gate_batch_rows(c, w.gate, B, &res, in, nin, d_var);
    rv.resize(B);
    for (int i = 0; i < B; ++i) {
        memcpy(&ra[(size_t)i * kn], recs[i].a, kn * 4);
        rb[i] = recs[i].b;
        rv[i] = recs[i].var;
    }
    return rc;
}

static bool same(const Work &w, const std::vector<int32_t> &ra, const std::vector<int32_t> &rb,
                 const std::vector<double> &rv) {
    if (ra != w.want_a || rb != w.want_b) return false;
    if (w.path == RECORDS && (rv.size() != w.want_v.size() || memcmp(rv.data(), w.want_v.data(), rv.size() * 8)))
        return false;
    return true;
}

int main(int argc, char **argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 8;
    const int reps = argc > 2 ? atoi(argv[2]) : 2;
    hip_stub::device_count() = 2;
    // keys: their content is irrelevant to the stand-in kernels, but they are uploaded and copied
    std::vector<int32_t> bk((size_t)500 * 4 * 2 * 1024), ksk((size_t)1024 * 8 * 4 * 501);
    uint32_t s = 99;
    for (auto &x : bk) x = (int32_t)lcg(s);
    for (auto &x : ksk) x = (int32_t)lcg(s);
    TfheAmdContext *c0 = nullptr, *c1 = nullptr, *c2 = nullptr;
    CHECK(tfhe_amd_context_create_raw(bk.data(), ksk.data(), 0, &c0) == 0, "context 0");
    CHECK(tfhe_amd_context_create_raw(bk.data(), ksk.data(), 1, &c1) == 0, "context 1");
    if (g_fail) return 1;
    double *d_var = nullptr;   // the KSK row variances [1024][8][4] the record path reads on the device
    CHECK(tfhe_amd_internal_upload(c0, std::vector<double>(1024 * 8 * 4, 1e-9).data(), 1024 * 8 * 4 * 8,
                                   (void **)&d_var) == 0, "upload");

    // workloads: (gate, B, path)
    const int shapes[][3] = {{TFHE_GATE_NAND, 64, STAGED},   {TFHE_GATE_AND, 700, STAGED},
                             {TFHE_GATE_XOR, 1100, STAGED},  {TFHE_GATE_MUX, 2100, STAGED},
                             {TFHE_GATE_NAND, 64, PINNED},   {TFHE_GATE_OR, 700, PINNED},
                             {TFHE_GATE_MUX, 1100, PINNED},  {TFHE_GATE_NOR, 96, RECORDS},
                             {TFHE_GATE_XNOR, 1100, RECORDS}, {TFHE_GATE_MUX, 600, RECORDS}};
    std::vector<Work> works;
    for (size_t i = 0; i < sizeof shapes / sizeof shapes[0]; ++i) {
        Work w;
        w.gate = shapes[i][0];
        w.B = shapes[i][1];
        w.path = shapes[i][2];
        w.seed = 1000u + (uint32_t)i;
        make_inputs(w);
        works.push_back(std::move(w));
    }
    // sequential reference on context 0
    for (Work &w : works) {
        CHECK(run(c0, w, d_var, w.want_a, w.want_b, w.want_v) == 0, "sequential %s B=%d", kPath[w.path], w.B);
    }
    // the three host paths agree with each other on the same inputs (staged vs pinned vs records)
    {
        Work a = works[5];   // OR 700 pinned
        a.path = STAGED;
        std::vector<int32_t> ra, rb;
        std::vector<double> rv;
        CHECK(run(c0, a, d_var, ra, rb, rv) == 0 && ra == works[5].want_a && rb == works[5].want_b,
              "staged == pinned");
        a.path = RECORDS;
        CHECK(run(c0, a, d_var, ra, rb, rv) == 0 && ra == works[5].want_a && rb == works[5].want_b,
              "records == pinned");
    }
    printf("sequential: %zu workloads\n", works.size());

    // phase 1: T threads over three contexts, several on one context; the replica is built meanwhile
    std::atomic<int> mism{0}, calls{0};
    std::thread replica([&] {
        CHECK(tfhe_amd_context_create_replica(c0, 1, &c2) == 0, "replica");
    });
    {
        std::vector<std::thread> ts;
        for (int t = 0; t < threads; ++t)
            ts.emplace_back([&, t] {
                std::vector<int32_t> ra, rb;
                std::vector<double> rv;
                for (int r = 0; r < reps; ++r)
                    for (size_t i = 0; i < works.size(); ++i) {
                        const Work &w = works[(i + (size_t)t * 3) % works.size()];
                        TfheAmdContext *c = (t % 3 == 2) ? c1 : c0;   // 2 of 3 threads share context 0
                        if (run(c, w, d_var, ra, rb, rv) != 0) {
                            CHECK(false, "thread %d %s B=%d failed", t, kPath[w.path], w.B);
                            continue;
                        }
                        calls++;
                        if (!same(w, ra, rb, rv)) mism++;
                    }
            });
        replica.join();
        for (auto &th : ts) th.join();
    }
    CHECK(mism == 0, "phase 1: %d of %d results differ from the sequential run", mism.load(), calls.load());
    printf("engine host paths: %d threads x %d reps, %d calls over 3 contexts, all equal\n", threads, reps,
           calls.load());

    // the replica serves the same results
    {
        std::vector<int32_t> ra, rb;
        std::vector<double> rv;
        for (int i : {2, 6}) {
            CHECK(c2 && run(c2, works[i], d_var, ra, rb, rv) == 0 && same(works[i], ra, rb, rv), "replica %d", i);
        }
    }

    // phase 2: registry churn beside pinned batches
    {
        std::atomic<bool> stop{false};
        std::atomic<int> churn{0};
        std::vector<std::thread> ts;
        for (int t = 0; t < 2; ++t)
            ts.emplace_back([&] {
                std::vector<void *> held;
                while (!stop) {
                    void *p = tfhe_amd_host_alloc(4096);
                    CHECK(p && tfhe_amd_host_is_pinned(p, 4096) == 1, "alloc");
                    held.push_back(p);
                    if (held.size() > 8) {
                        CHECK(tfhe_amd_host_free(held.front()) == 0, "free");
                        held.erase(held.begin());
                    }
                    churn++;
                }
                for (void *p : held) tfhe_amd_host_free(p);
            });
        std::vector<int32_t> ra, rb;
        std::vector<double> rv;
        for (int r = 0; r < 3; ++r)
            for (int i : {4, 5, 6}) {
                CHECK(run(c1, works[i], d_var, ra, rb, rv) == 0 && same(works[i], ra, rb, rv), "phase 2 %d", i);
            }
        stop = true;
        for (auto &th : ts) th.join();
        printf("pinned registry: %d alloc/free beside pinned batches\n", churn.load());
    }

    tfhe_amd_internal_free(0, d_var);
    CHECK(tfhe_amd_context_destroy(c2) == 0 && tfhe_amd_context_destroy(c1) == 0 && tfhe_amd_context_destroy(c0) == 0,
          "destroy");
    if (g_fail) return 1;
    printf("tsan_engine_driver: ok\n");
    return 0;
}
