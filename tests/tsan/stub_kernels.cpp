// Test-only CPU stand-ins for the HIP kernels' launchers (csrc/*.hip), so that csrc/engine.cpp itself
// — the host copy pool, the pinned registry, the sliced / record / pinned host paths, the context
// lock, replicas — builds against the stub HIP runtime (stub/hip/hip_runtime.h) and runs under
// ThreadSanitizer (tests/tsan/tsan_engine_driver.cpp, tests/test_concurrency_tsan.py).  Each
// launcher enqueues its work on the stream it is given, like a kernel launch: it runs later on that
// stream's worker thread, so the engine's stream / event ordering is what makes its results visible
// to the host.  The arithmetic is a deterministic stand-in (not TFHE): every output word is a hash
// of the inputs the real kernel would read, so a concurrent run can be compared word for word with
// a sequential one.  Not product code.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "engine.h"

namespace tfhe_amd {
namespace {

uint32_t mix(uint32_t x, uint32_t k) {
    x ^= k * 0x9E3779B9u;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    return x * 0xC2B2AE35u;
}

// the "blind rotation" of one linear combination x = (0, c) + sa X + sb Y + sc Z -> u (N + 1 words)
void fake_br(const int32_t *xa, int32_t xb, int32_t sa, const int32_t *ya, int32_t yb, int32_t sb, const int32_t *za,
             int32_t zb, int32_t sc, int32_t c, int32_t mu, int32_t *u_a, int32_t *u_b) {
    uint32_t lin[kn];
    for (int j = 0; j < kn; ++j) {
        uint32_t v = (uint32_t)sa * (uint32_t)xa[j];
        if (ya) v += (uint32_t)sb * (uint32_t)ya[j];
        if (za) v += (uint32_t)sc * (uint32_t)za[j];
        lin[j] = v;
    }
    uint32_t b = (uint32_t)c + (uint32_t)sa * (uint32_t)xb + (ya ? (uint32_t)sb * (uint32_t)yb : 0u) +
                 (za ? (uint32_t)sc * (uint32_t)zb : 0u);
    for (int j = 0; j < kN; ++j) u_a[j] = (int32_t)mix(lin[j % kn] + (uint32_t)j, (uint32_t)mu ^ b);
    *u_b = (int32_t)mix(b, (uint32_t)mu);
}

// the "key switch" of u (+ u2) + (0, add_b) -> res (n + 1 words)
void fake_ks(const int32_t *ua, int32_t ub, const int32_t *u2a, const int32_t *u2b, int32_t add_b, int32_t *ra,
             int32_t *rb) {
    for (int j = 0; j < kn; ++j) {
        uint32_t v = (uint32_t)ua[j] + (j + kn < kN ? (uint32_t)ua[j + kn] : 0u);
        if (u2a) v += (uint32_t)u2a[j];
        ra[j] = (int32_t)mix(v, 3u);
    }
    *rb = (int32_t)((uint32_t)ub + (u2b ? (uint32_t)*u2b : 0u) + (uint32_t)add_b);
}

}  // namespace

hipError_t launch_bk_to_ntt(const int32_t *, uint32_t *, const NttTables *, hipStream_t) { return hipSuccess; }
void build_v2_twiddles(const NttTables &, uint2 *, uint2 *, uint2 *, uint2 *) {}
hipError_t launch_bk_v1_to_v2(const uint32_t *, uint32_t *, hipStream_t) { return hipSuccess; }
void build_v4_twiddles(const NttTables &, uint2 *, uint2 *, uint2 *) {}
void build_v6_twiddles(double2 *) {}
hipError_t launch_bk_to_fft(const int32_t *, double2 *, const double2 *, hipStream_t) { return hipSuccess; }
hipError_t launch_ksk_to_v5(const int32_t *, int32_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_ksk_to_v4(const int32_t *, int32_t *, hipStream_t) { return hipSuccess; }
int ks_version() { return 5; }
size_t ksk_v4_words() { return 64; }
size_t ksk_v5_words() { return 64; }
bool ks5_enabled() { return true; }

static hipError_t br(int B, int halves, const BrInput *in, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t s,
                     const Guard *guard) {
    const BrInput i0 = in[0], i1 = halves > 1 ? in[1] : in[0];
    uint32_t *flags = guard ? guard->flags : nullptr;
    hip_stub::enqueue(s, [=] {
        for (int g = 0; g < B * halves; ++g) {
            const BrInput &x = g < B ? i0 : i1;
            const int k = g < B ? g : g - B;
            fake_br(x.x_a + (size_t)k * kn, x.x_b[k], x.sa, x.sb ? x.y_a + (size_t)k * kn : nullptr,
                    x.sb ? x.y_b[k] : 0, x.sb, nullptr, 0, 0, x.c, mu, u_a + (size_t)g * kN, u_b + g);
            if (flags) flags[2 * g] = flags[2 * g + 1] = 0;   // nothing for the guard to recompute
        }
    });
    return hipSuccess;
}
hipError_t launch_blind_rotate_v6(const DeviceKey &, int B, int halves, const BrInput *in, int32_t mu, int32_t *u_a,
                                  int32_t *u_b, hipStream_t s, const Guard *guard) {
    trace_kernel("stub_blind_rotate");
    return br(B, halves, in, mu, u_a, u_b, s, guard);
}
hipError_t launch_blind_rotate_v4(const DeviceKey &, int B, int halves, const BrInput *in, int32_t mu, int32_t *u_a,
                                  int32_t *u_b, hipStream_t s, const Guard *guard) {
    if (guard) {   // guard mode: reads the flags the v6 stand-in wrote (all clear), recomputes nothing
        const uint32_t *flags = guard->flags;
        hip_stub::enqueue(s, [=] {
            volatile uint32_t acc = 0;
            for (int g = 0; g < B * halves; ++g) acc = acc | flags[2 * g] | flags[2 * g + 1];
            (void)acc;
        });
        return hipSuccess;
    }
    return br(B, halves, in, mu, u_a, u_b, s, nullptr);
}

static hipError_t br_rows(int B, int nrows, const CircRow *rows, const int32_t *wa, const int32_t *wb, int32_t mu,
                          int32_t *u_a, int32_t *u_b, hipStream_t s, const Guard *guard) {
    uint32_t *flags = guard ? guard->flags : nullptr;
    hip_stub::enqueue(s, [=] {
        for (int r = 0; r < nrows; ++r) {
            const CircRow row = rows[r];
            for (int k = 0; k < B; ++k) {
                auto wire = [&](int w, const int32_t *&a, int32_t &b) {
                    a = w >= 0 ? wa + ((size_t)w * B + k) * kn : nullptr;
                    b = w >= 0 ? wb[(size_t)w * B + k] : 0;
                };
                const int32_t *xa, *ya, *za;
                int32_t xb, yb, zb;
                wire(row.x, xa, xb);
                wire(row.y, ya, yb);
                wire(row.z, za, zb);
                const size_t slot = (size_t)r * B + k;
                fake_br(xa, xb, row.sa, ya, yb, row.sb, za, zb, row.sc, row.c, mu, u_a + slot * kN, u_b + slot);
                if (flags) flags[2 * slot] = flags[2 * slot + 1] = 0;
            }
        }
    });
    return hipSuccess;
}
hipError_t launch_blind_rotate_v4_rows(const DeviceKey &, int B, int nrows, const CircRow *rows, const int32_t *wa,
                                       const int32_t *wb, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t s,
                                       const Guard *guard) {
    if (guard) return hipSuccess;
    return br_rows(B, nrows, rows, wa, wb, mu, u_a, u_b, s, nullptr);
}
hipError_t launch_blind_rotate_v6_rows(const DeviceKey &, int B, int nrows, const CircRow *rows, const int32_t *wa,
                                       const int32_t *wb, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t s,
                                       const Guard *guard) {
    trace_kernel("stub_blind_rotate_rows");
    return br_rows(B, nrows, rows, wa, wb, mu, u_a, u_b, s, guard);
}
hipError_t launch_blind_rotate_v4_debug(const DeviceKey &, int, int, int32_t *, const int32_t *, hipStream_t) {
    return hipSuccess;
}
hipError_t launch_blind_rotate_v6_debug(const DeviceKey &, int, int, int32_t *, const int32_t *, hipStream_t) {
    return hipSuccess;
}
hipError_t launch_external_product_v4(const DeviceKey &, int, const int32_t *, int32_t *, hipStream_t) {
    return hipSuccess;
}

hipError_t launch_keyswitch(const DeviceKey &, int B, const int32_t *u_a, const int32_t *u_b, const int32_t *u2_a,
                            const int32_t *u2_b, int32_t add_b, int32_t *res_a, int32_t *res_b, hipStream_t s) {
    trace_kernel("stub_keyswitch");
    hip_stub::enqueue(s, [=] {
        for (int i = 0; i < B; ++i)
            fake_ks(u_a + (size_t)i * kN, u_b[i], u2_a ? u2_a + (size_t)i * kN : nullptr, u2_b ? u2_b + i : nullptr,
                    add_b, res_a + (size_t)i * kn, res_b + i);
    });
    return hipSuccess;
}
hipError_t launch_keyswitch_rows(const DeviceKey &, int B, int nks, const CircKs *ks, const int32_t *u_a,
                                 const int32_t *u_b, int32_t *wa, int32_t *wb, hipStream_t s) {
    hip_stub::enqueue(s, [=] {
        for (int g = 0; g < nks; ++g) {
            const CircKs e = ks[g];
            for (int k = 0; k < B; ++k) {
                const size_t r1 = (size_t)e.r1 * B + k, r2 = (size_t)e.r2 * B + k, o = (size_t)e.out * B + k;
                fake_ks(u_a + r1 * kN, u_b[r1], e.r2 >= 0 ? u_a + r2 * kN : nullptr, e.r2 >= 0 ? u_b + r2 : nullptr,
                        e.add_b, wa + o * kn, wb + o);
            }
        }
    });
    return hipSuccess;
}
hipError_t launch_circuit_linear(int B, int nlin, const CircLin *lin, int32_t *wa, int32_t *wb, hipStream_t s) {
    hip_stub::enqueue(s, [=] {
        for (int g = 0; g < nlin; ++g) {
            const CircLin e = lin[g];
            for (int k = 0; k < B; ++k) {
                const size_t o = (size_t)e.out * B + k;
                for (int j = 0; j < kn; ++j)
                    wa[o * kn + j] = e.in >= 0 ? (int32_t)((uint32_t)e.s * (uint32_t)wa[((size_t)e.in * B + k) * kn + j]) : 0;
                wb[o] = (int32_t)((uint32_t)e.c + (e.in >= 0 ? (uint32_t)e.s * (uint32_t)wb[(size_t)e.in * B + k] : 0u));
            }
        }
    });
    return hipSuccess;
}
static double fake_var(const int32_t *u) { return (double)((uint32_t)u[0] & 0xffffu) * 1e-9 + 1e-6; }
hipError_t launch_ks_variance(const int32_t *u_a, int B, int halves, const double *, double *out, hipStream_t s) {
    hip_stub::enqueue(s, [=] {
        for (int i = 0; i < B; ++i)
            out[i] = fake_var(u_a + (size_t)i * kN) + (halves > 1 ? fake_var(u_a + ((size_t)B + i) * kN) : 0.0);
    });
    return hipSuccess;
}
hipError_t launch_ks_variance_rows(const int32_t *u_a, int B, const CircKs *ks, const double *, double *out,
                                   hipStream_t s) {
    hip_stub::enqueue(s, [=] {
        for (int i = 0; i < B; ++i) {
            const CircKs e = ks[i];
            out[i] = fake_var(u_a + (size_t)e.r1 * kN) + (e.r2 >= 0 ? fake_var(u_a + (size_t)e.r2 * kN) : 0.0);
        }
    });
    return hipSuccess;
}

}  // namespace tfhe_amd

// ceiling.hip's measurement is GPU-only
extern "C" int tfhe_amd_fp64_ceiling(int, int, double, double *, double *) { return -3; }
