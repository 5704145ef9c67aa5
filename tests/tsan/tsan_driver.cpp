// ThreadSanitizer driver for the library's concurrency code (tests/test_concurrency_tsan.py):
// tfhe_api.cpp (key registry, per-thread lanes, the two-lane Tier-1 coalescing queue),
// multi.cpp (tfhe_gpu_init registry, per-device workers) and circuit.cpp (per-context device
// state, dropped with its context) built with -fsanitize=thread against the CPU stand-in engine
// (stub_engine.cpp) and the HIP stand-in header (stub/hip/hip_runtime.h).  Every phase compares
// its concurrent results word for word (and current_variance bit for bit) with the same work run
// sequentially.  Exit 0 = all equal; ThreadSanitizer itself exits 66 on any report.
// Reference callers whose concurrency this models: cpuParallel/Cipher.cpp:83-120 (OpenMP gate
// calls, results aliasing inputs), cloud.cpp:389-395; the reference's own engine is not
// reentrant (gpuParallel/lagrangehalfc_impl.cu:4).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "engine.h"
#include "../../include/tfhe/tfhe.h"
#include "../../include/tfhe/tfhe_io.h"
#include "../../include/tfhe_amd.h"

extern "C" long stub_live_contexts();
extern "C" long stub_set_device_calls();

static int g_fail = 0;
#define CHECK(cond, ...)                                    \
    do {                                                    \
        if (!(cond)) {                                      \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                   \
            fprintf(stderr, "\n");                          \
            g_fail = 1;                                     \
        }                                                   \
    } while (0)

using tfhe_amd::DeviceScope;

// ---- DeviceScope (engine.h): save / switch / restore, nesting, no-op cases
static void test_device_scope() {
    hipSetDevice(1);
    const long calls0 = stub_set_device_calls();
    {
        DeviceScope a(0);
        int d = -1;
        hipGetDevice(&d);
        CHECK(d == 0 && a.rc == hipSuccess, "scope(0) from 1: current %d", d);
        {
            DeviceScope b(1);
            hipGetDevice(&d);
            CHECK(d == 1, "nested scope(1): current %d", d);
        }
        hipGetDevice(&d);
        CHECK(d == 0, "after nested scope: current %d", d);
        {
            DeviceScope same(0);   // already current: no hipSetDevice
            DeviceScope none(-1);  // no device: no switch
            hipGetDevice(&d);
            CHECK(d == 0, "no-op scopes: current %d", d);
        }
    }
    int d = -1;
    hipGetDevice(&d);
    CHECK(d == 1, "caller's device restored: current %d", d);
    // 3 switches: into 0, into nested 1, back to 0 (nested restore), back to 1 (outer restore)
    CHECK(stub_set_device_calls() - calls0 == 4, "hipSetDevice calls %ld", stub_set_device_calls() - calls0);
    {
        DeviceScope bad(7);   // a device that does not exist: rc reports it, nothing changes
        hipGetDevice(&d);
        CHECK(bad.rc != hipSuccess && d == 1, "invalid device: rc %d current %d", (int)bad.rc, d);
    }
    hipSetDevice(0);
}

struct Ct {   // one ciphertext, compared by value
    std::vector<int32_t> a;
    int32_t b;
    double var;
};
static Ct snap(const LweSample *s) { return Ct{std::vector<int32_t>(s->a, s->a + 500), s->b, s->current_variance}; }
static bool same(const Ct &x, const Ct &y) { return x.a == y.a && x.b == y.b && memcmp(&x.var, &y.var, 8) == 0; }

// ---- Tier-1: a per-thread chain of gates over the thread's own ciphertexts, results aliasing
// inputs, mixed kinds (incl. MUX) so that the queue's batches mix gate kinds
static const int kGates[] = {TFHE_GATE_NAND, TFHE_GATE_XOR, TFHE_GATE_AND, TFHE_GATE_MUX, TFHE_GATE_ORYN,
                             TFHE_GATE_XNOR, TFHE_GATE_NOR, TFHE_GATE_ANDNY, TFHE_GATE_OR, TFHE_GATE_ORNY};
static void gate_call(int g, LweSample *r, const LweSample *a, const LweSample *b, const LweSample *c,
                      const TFheGateBootstrappingCloudKeySet *bk) {
    switch (g) {
    case TFHE_GATE_NAND: bootsNAND(r, a, b, bk); break;
    case TFHE_GATE_XOR: bootsXOR(r, a, b, bk); break;
    case TFHE_GATE_AND: bootsAND(r, a, b, bk); break;
    case TFHE_GATE_MUX: bootsMUX(r, a, b, c, bk); break;
    case TFHE_GATE_ORYN: bootsORYN(r, a, b, bk); break;
    case TFHE_GATE_XNOR: bootsXNOR(r, a, b, bk); break;
    case TFHE_GATE_NOR: bootsNOR(r, a, b, bk); break;
    case TFHE_GATE_ANDNY: bootsANDNY(r, a, b, bk); break;
    case TFHE_GATE_OR: bootsOR(r, a, b, bk); break;
    default: bootsORNY(r, a, b, bk); break;
    }
}
struct Chain {
    LweSample *v;   // 4 ciphertexts
    int seed;
};
static void run_chain(Chain &c, int steps, const TFheGateBootstrappingCloudKeySet *bk) {
    for (int s = 0; s < steps; ++s) {
        const int g = kGates[(c.seed + 3 * s) % 10];
        const int r = (c.seed + s) % 4, x = (c.seed + 2 * s + 1) % 4, y = (c.seed + s + 2) % 4, z = (s + 3) % 4;
        // r often equals x or y: the result aliases an input (Cipher.cpp:387 bootsAND(t1, t1, t2))
        gate_call(g, &c.v[r], &c.v[x], &c.v[y], &c.v[z], bk);
    }
}

static void fill(LweSample *s, int seed) {
    uint32_t x = 2463534242u + 977u * (uint32_t)seed;
    for (int j = 0; j < 500; ++j) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        s->a[j] = (int32_t)x;
    }
    s->b = (int32_t)(x * 2654435761u);
    s->current_variance = 0;
}

static void test_tier1(const TFheGateBootstrappingParameterSet *params, const TFheGateBootstrappingCloudKeySet *bk,
                       int threads, int steps) {
    std::vector<Chain> seq(threads), par(threads);
    for (int t = 0; t < threads; ++t) {
        seq[t] = Chain{new_gate_bootstrapping_ciphertext_array(4, params), t};
        par[t] = Chain{new_gate_bootstrapping_ciphertext_array(4, params), t};
        for (int k = 0; k < 4; ++k) {
            fill(&seq[t].v[k], 4 * t + k);
            fill(&par[t].v[k], 4 * t + k);
        }
    }
    for (int t = 0; t < threads; ++t) run_chain(seq[t], steps, bk);   // one thread: B = 1 batches
    long long b0, g0, m0;
    tfhe_amd_tier1_queue_stats(bk, &b0, &g0, &m0, 1);
    std::vector<std::thread> th;
    std::atomic<int> go{0};
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            while (!go.load()) std::this_thread::yield();
            run_chain(par[t], steps, bk);
        });
    go = 1;
    for (auto &x : th) x.join();
    long long batches, gates, largest;
    tfhe_amd_tier1_queue_stats(bk, &batches, &gates, &largest, 0);
    int bad = 0;
    for (int t = 0; t < threads; ++t)
        for (int k = 0; k < 4; ++k) bad += !same(snap(&seq[t].v[k]), snap(&par[t].v[k]));
    CHECK(bad == 0, "tier1: %d of %d ciphertexts differ from the sequential run", bad, 4 * threads);
    CHECK(gates == (long long)threads * steps, "tier1: queue ran %lld gates, expected %d", gates, threads * steps);
    printf("tier1: %d threads x %d gates: %lld batches (largest %lld), all equal to sequential\n", threads, steps,
           batches, largest);
    for (int t = 0; t < threads; ++t) {
        delete_gate_bootstrapping_ciphertext_array(4, seq[t].v);
        delete_gate_bootstrapping_ciphertext_array(4, par[t].v);
    }
}

// ---- LweSample-array batches (tfhe_amd_boots_batch) from several threads, each on its own arrays
// (one in place: result = input a; one of two slices), against the single-gate calls one by one
static void test_boots_batch(const TFheGateBootstrappingParameterSet *params, const TFheGateBootstrappingCloudKeySet *bk,
                             int threads) {
    const int sizes[] = {1, 7, 64, 1100};
    std::vector<LweSample *> a(threads), b(threads), c(threads), r(threads), ref(threads);
    std::vector<int> n(threads), g(threads);
    for (int t = 0; t < threads; ++t) {
        n[t] = sizes[t % 4];
        g[t] = kGates[t % 10];
        a[t] = new_gate_bootstrapping_ciphertext_array(n[t], params);
        b[t] = new_gate_bootstrapping_ciphertext_array(n[t], params);
        c[t] = new_gate_bootstrapping_ciphertext_array(n[t], params);
        r[t] = new_gate_bootstrapping_ciphertext_array(n[t], params);
        ref[t] = new_gate_bootstrapping_ciphertext_array(n[t], params);
        for (int i = 0; i < n[t]; ++i) {
            fill(&a[t][i], 7000 + 3 * i + t);
            fill(&b[t][i], 9000 + 5 * i + t);
            fill(&c[t][i], 11000 + 7 * i + t);
            gate_call(g[t], &ref[t][i], &a[t][i], &b[t][i], &c[t][i], bk);
        }
    }
    std::vector<std::thread> th;
    std::vector<int> rcs(threads, 0);
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            LweSample *out = t % 3 == 0 ? a[t] : r[t];   // in place on every third thread
            rcs[t] = tfhe_amd_boots_batch(g[t], out, a[t], b[t], c[t], n[t], bk);
        });
    for (auto &x : th) x.join();
    int bad = 0, badv = 0;
    for (int t = 0; t < threads; ++t) {
        CHECK(rcs[t] == TFHE_AMD_OK, "boots_batch: thread %d rc %d", t, rcs[t]);
        const LweSample *out = t % 3 == 0 ? a[t] : r[t];
        for (int i = 0; i < n[t]; ++i) {
            bad += !same(snap(&out[i]), snap(&ref[t][i]));
            badv += out[i].current_variance != ref[t][i].current_variance;
        }
    }
    CHECK(bad == 0 && badv == 0, "boots_batch: %d results and %d variances differ from single gates", bad, badv);
    printf("boots_batch: %d threads (sizes 1-1100, in place on every third), equal to single gates\n", threads);
    for (int t = 0; t < threads; ++t)
        for (LweSample *x : {a[t], b[t], c[t], r[t], ref[t]}) delete_gate_bootstrapping_ciphertext_array(n[t], x);
}

// ---- Tier-2 multi-device registry: tfhe_gpu_boots_batch on a key while tfhe_gpu_init
// re-registers it, and other keys are imported, registered, used and deleted
static void soa(int B, int seed, std::vector<int32_t> &a, std::vector<int32_t> &b) {
    a.resize((size_t)B * 500);
    b.resize(B);
    uint32_t x = 88172645u + 31u * (uint32_t)seed;
    for (auto &v : a) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v = (int32_t)x; }
    for (auto &v : b) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v = (int32_t)x; }
}
static void test_multi(const TFheGateBootstrappingCloudKeySet *bk, const std::string &cloud_bytes, int threads) {
    const int B = 37;
    std::vector<int32_t> xa, xb, ya, yb;
    soa(B, 1, xa, xb);
    soa(B, 2, ya, yb);
    std::vector<int32_t> wa((size_t)B * 500), wb(B);
    CHECK(tfhe_gpu_boots_batch(TFHE_GATE_XOR, wa.data(), wb.data(), xa.data(), xb.data(), ya.data(), yb.data(),
                               nullptr, nullptr, B, bk) == 0, "tier-1 fallback batch");
    std::atomic<bool> stop{false};
    std::atomic<int> bad{0}, runs{0};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            hipSetDevice(t & 1);   // callers on either device keep theirs
            std::vector<int32_t> ra((size_t)B * 500), rb(B);
            while (!stop.load()) {
                if (tfhe_gpu_boots_batch(TFHE_GATE_XOR, ra.data(), rb.data(), xa.data(), xb.data(), ya.data(),
                                         yb.data(), nullptr, nullptr, B, bk) != 0 ||
                    ra != wa || rb != wb)
                    bad++;
                int d = -1;
                hipGetDevice(&d);
                if (d != (t & 1)) bad++;
                runs++;
            }
        });
    std::thread reg([&] {   // re-registration of the key in use
        for (int i = 0; i < 6; ++i) CHECK(tfhe_gpu_init(bk, i & 1 ? 3 : 1) == 0, "tfhe_gpu_init");
    });
    std::thread churn([&] {   // other keys come and go
        for (int i = 0; i < 2; ++i) {
            std::istringstream in(cloud_bytes);
            TFheGateBootstrappingCloudKeySet *k2 = new_tfheGateBootstrappingCloudKeySet_fromStream(in);
            CHECK(tfhe_gpu_init(k2, 3) == 0, "tfhe_gpu_init(k2)");
            std::vector<int32_t> ra((size_t)B * 500), rb(B);
            CHECK(tfhe_gpu_boots_batch(TFHE_GATE_XOR, ra.data(), rb.data(), xa.data(), xb.data(), ya.data(), yb.data(),
                                       nullptr, nullptr, B, k2) == 0 && ra == wa && rb == wb, "k2 batch");
            LweSample *c = new_gate_bootstrapping_ciphertext_array(3, k2->params);
            for (int k = 0; k < 3; ++k) fill(&c[k], 100 + k);
            bootsAND(&c[0], &c[1], &c[2], k2);   // its Tier-1 context and queue
            delete_gate_bootstrapping_ciphertext_array(3, c);
            delete_gate_bootstrapping_cloud_keyset(k2);
        }
    });
    reg.join();
    churn.join();
    stop = true;
    for (auto &x : th) x.join();
    CHECK(bad.load() == 0, "multi: %d of %d concurrent batches wrong (or the caller's device moved)", bad.load(),
          runs.load());
    printf("multi: %d concurrent tfhe_gpu_boots_batch calls during re-registration and key churn, all equal\n",
           runs.load());
}

// ---- circuits: one circuit run concurrently on several contexts while others come and go
static void test_circuits(const TFheGateBootstrappingCloudKeySet *bk, int threads) {
    TfheAmdCircuit *C = nullptr;
    tfhe_amd_circuit_create(&C);
    int a[8], b[8], s[8];
    const int first = tfhe_amd_circuit_inputs(C, 16);
    for (int i = 0; i < 8; ++i) { a[i] = first + i; b[i] = first + 8 + i; }
    tfhe_amd_circuit_add(C, 8, a, b, -1, s);
    int nw = 0, ng = 0, nb = 0, depth = 0;
    tfhe_amd_circuit_info(C, &nw, &ng, &nb, &depth);
    const int B = 5;
    std::vector<int32_t> wa0((size_t)nw * B * 500), wb0((size_t)nw * B);
    uint32_t x = 12345;
    for (int i = 0; i < 16 * B * 500; ++i) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; wa0[(size_t)first * B * 500 + i] = (int32_t)x; }
    for (int i = 0; i < 16 * B; ++i) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; wb0[(size_t)first * B + i] = (int32_t)x; }
    std::vector<int32_t> want_a = wa0, want_b = wb0;
    {
        TfheAmdContext *c0 = nullptr;
        tfhe_amd_context_create(bk, 0, &c0);
        CHECK(tfhe_amd_circuit_run_dev(c0, C, B, want_a.data(), want_b.data(), nullptr) == 0, "circuit run");
        tfhe_amd_context_destroy(c0);
    }
    CHECK(tfhe_amd_circuit_state_count(C) == 0, "state dropped with its context: %d left",
          tfhe_amd_circuit_state_count(C));
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            for (int rep = 0; rep < 3; ++rep) {
                TfheAmdContext *c = nullptr;
                if (tfhe_amd_context_create(bk, t & 1, &c) != 0) { bad++; continue; }
                std::vector<int32_t> wa = wa0, wb = wb0;
                if (tfhe_amd_circuit_run_dev(c, C, B, wa.data(), wb.data(), nullptr) != 0 || wa != want_a ||
                    wb != want_b)
                    bad++;
                tfhe_amd_context_destroy(c);
            }
        });
    for (auto &t : th) t.join();
    CHECK(bad.load() == 0, "circuits: %d concurrent runs wrong", bad.load());
    CHECK(tfhe_amd_circuit_state_count(C) == 0, "circuits: %d states left after their contexts",
          tfhe_amd_circuit_state_count(C));
    tfhe_amd_circuit_destroy(C);
    printf("circuits: %d threads x 3 contexts, one shared circuit, results equal, no state left\n", threads);
}

int main(int argc, char **argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 64;
    const int steps = argc > 2 ? atoi(argv[2]) : 8;
    hip_stub::device_count() = 2;
    test_device_scope();
    TFheGateBootstrappingParameterSet *params = new_default_gate_bootstrapping_parameters(110);
    uint32_t seed[] = {314, 1592, 657};
    tfhe_random_generator_setSeed(seed, 3);
    TFheGateBootstrappingSecretKeySet *key = new_random_gate_bootstrapping_secret_keyset(params);
    const TFheGateBootstrappingCloudKeySet *bk = &key->cloud;
    std::ostringstream out;
    export_tfheGateBootstrappingCloudKeySet_toStream(out, bk);
    const std::string cloud_bytes = out.str();
    test_tier1(params, bk, threads, steps);
    test_boots_batch(params, bk, 8);
    test_multi(bk, cloud_bytes, 8);
    test_circuits(bk, 8);
    delete_gate_bootstrapping_secret_keyset(key);
    delete_gate_bootstrapping_parameters(params);
    CHECK(stub_live_contexts() == 0, "%ld contexts leaked", stub_live_contexts());
    printf(g_fail ? "tsan_driver: FAILED\n" : "tsan_driver: ok\n");
    return g_fail;
}
