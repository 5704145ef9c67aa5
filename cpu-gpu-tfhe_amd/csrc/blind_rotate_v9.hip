// blind_rotate_v9.hip — blind rotation with 4 waves per ciphertext, for launches of at most two
// ciphertexts per CU (B <= 512 on 256 CUs: the 8-GPU strong-scaled 4 096, circuit levels, the
// Tier-1 queue's batches and single gates).
//
// v6 gives a ciphertext 2 waves, so B = 512 leaves one wave per SIMD (and B <= 256 leaves half
// the SIMDs idle): a lone wave cannot issue fp64 back to back (0.77 of the two-wave rate,
// DESIGN.md §5.1) and every LDS round trip and barrier of its step is exposed.  Here the step's
// work is split four ways, evenly, so that two ciphertexts per CU put two waves on every SIMD:
//
//  * wave q = (w, d) = (q >> 1, q & 1) holds accumulator polynomial w (its 16 Torus32
//    coefficients per lane, layout A: j = L + 64 r) — both waves of a pair hold the same copy —,
//    rotates it in registers (ds_bpermute), takes gadget digit d of (X^a - 1) ACC_w (TGSW row
//    2w + d, tgsw-functions.cu:300-413) and runs v6's forward transform of that ONE digit
//    polynomial (fft_wave.h: passes A, B, C), whose spectrum it stores to its LDS buffer;
//  * barrier; wave q = (c, h) then MACs the four spectra over half h of the slots of output c
//    (slot s = 256 h + 4 L + t, t < 4) with the key rows (tgsw-fft-operations.cu:124-264; the key
//    re-laid per (c, h) so that each of the 16 loads is 1 KB contiguous) and runs the DIT stages
//    0..7 of its half as four radix-4 register passes (layouts P, Q, R, S: register bits = slot
//    bits 0-1, 2-3, 4-5, 6-7) joined by three LDS transposes (slot map s ^ ((s >> 2) & 7):
//    conflict-free for all four layouts);
//  * the two waves of output c exchange their halves (h = 1 sends W_8 zeta^-L U1, h = 0 sends
//    zeta^-L U0) — barrier — and BOTH compute the whole output: stage 8, the register part of the
//    post-twist, rint -> acc_c (so each wave of a pair keeps the full accumulator polynomial).
// Per wave-step: one forward transform and half an inverse instead of two and one; two barriers.
// scripts/emu_v9.py emulates this data flow against the exact product; results are rounded to
// the exact integers like v6's and guarded the same way (flags of wave h = 0 of each output).
#include <cmath>
#include <cstdlib>
#include <vector>
#include "engine.h"
#include "modarith.h"
#include "fft_wave.h"

namespace tfhe_amd {

namespace {

constexpr int kV9Threads = 256;
constexpr int kTSlots = 256;   // a half spectrum (4 complex per lane), XOR-swizzled, no padding

struct __attribute__((aligned(16))) V9Shared {
    double2 S[4][kXSlots];     // per wave: forward transposes, then its spectrum (slot s at 9 (s >> 3) + (s & 7))
    double2 T[4][kTSlots];     // per wave: inverse transposes, then its half for the stage-8 exchange
    short bara[512];
    int barb;
};
static_assert(sizeof(V9Shared) <= 80 * 1024, "two v9 workgroups per CU");

struct V9Args {
    const double2 *bk9;   // [kn][2 c][2 h][4 rows][4 t][64 L]: FFT-domain key / 512, slot 256 h + 4 L + t
    const double2 *tw;    // build_v6_twiddles' table (forward passes)
    const double2 *tw9;   // build_v9_twiddles' table (inverse stages 2..7, post-twist lane factors)
    uint32_t *flags;      // exactness guard (engine.h Guard): [2 slot + w], or null
    uint32_t *stats;
};

// slot map of the inverse transposes (bank-conflict free for layouts P, Q, R and S)
__device__ __forceinline__ int tsw(int s) { return s ^ ((s >> 2) & 7); }
// local slot of (lane L, register t) in the inverse layouts
__device__ __forceinline__ int lay_P(int L, int t) { return 4 * L + t; }
__device__ __forceinline__ int lay_Q(int L, int t) { return (L & 3) + 4 * t + 16 * (L >> 2); }
__device__ __forceinline__ int lay_R(int L, int t) { return (L & 15) + 16 * t + 64 * (L >> 4); }
__device__ __forceinline__ int lay_S(int L, int t) { return L + 64 * t; }

// DIT stages k (register distance 1, twiddle a) and k + 1 (distance 2: b for register bit 0 = 0,
// -i b for 1): the two stages of a radix-4 register pass (emu_v9.radix4)
__device__ __forceinline__ void pass4(Cx (&x)[4], const Cx &a, const Cx &b) {
    bf_fwd<false>(x[0], x[1], a);
    bf_fwd<false>(x[2], x[3], a);
    bf_fwd<false>(x[0], x[2], b);
    bf_fwd<true>(x[1], x[3], negi_(b));
}
// stages 0 and 1: twiddles 1 and (1, -i)
__device__ __forceinline__ void pass4_first(Cx (&x)[4]) {
    bf_one(x[0], x[1]);
    bf_one(x[2], x[3]);
    bf_one(x[0], x[2]);
    bf_negi(x[1], x[3]);
}

template <int (*FROM)(int, int), int (*TO)(int, int)>
__device__ __forceinline__ void transpose4(double2 *T, Cx (&x)[4], int L) {
#pragma unroll
    for (int t = 0; t < 4; ++t) st(T + tsw(FROM(L, t)), x[t]);
    wave_sync();
#pragma unroll
    for (int t = 0; t < 4; ++t) x[t] = ld(T + tsw(TO(L, t)));
    wave_sync();
}

struct V9Tw {          // per-lane twiddles, held for the whole kernel
    Tw4 fB, fC;        // forward passes B and C (v6's table)
    Cx w2, w3, w4, w5, w6, w7;   // inverse DIT stages 2..7 (W_k(j) = e^{-i pi j / 2^k})
    Cx sc;             // h = 0: zeta^-L; h = 1: W_8(L) zeta^-L
};

// X^a ACC_w in registers (v6's RREG form): coefficient j = L + 64 r needs (j - a) mod 2N; with
// a = 64 q + s lane L takes lane (L - s) mod 64's register r - q (r - q - 1 for L < s) of the
// negacyclic ring of 32 registers; then the signed gadget digit d of (X^a - 1) ACC_w
__device__ __forceinline__ void rotate_digit(const uint32_t (&acc)[16], int a, int d, int L, Cx (&x)[8]) {
    const int aa = __builtin_amdgcn_readfirstlane(a) & (k2N - 1);
    const int s = aa & 63, q = aa >> 6;
    const int src = ((L - s) & 63) << 2;
    uint32_t V[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) V[r] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)acc[r]);
    if (q & 16) {
#pragma unroll
        for (int r = 0; r < 16; ++r) V[r] = 0u - V[r];
    }
#pragma unroll
    for (int K = 8; K >= 1; K >>= 1) {
        if (q & K) {
            uint32_t t[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) t[r] = r >= K ? V[r - K] : 0u - V[r + 16 - K];
#pragma unroll
            for (int r = 0; r < 16; ++r) V[r] = t[r];
        }
    }
    const bool lo = L < s;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t rot = lo ? (r ? V[r - 1] : 0u - V[15]) : V[r];
        const uint32_t diff = rot - acc[r];
        // hi = sext10 bits 22..31 of diff + off + 2^31, lo = sext10 bits 12..21 of diff + off + 2^21
        const int32_t dig = d == 0 ? (int32_t)(diff + (kDecompOffset + 0x80000000u)) >> 22
                                   : __builtin_amdgcn_sbfe((int32_t)(diff + (kDecompOffset + 0x200000u)), 12, 10);
        if (r < 8) x[r].re = (double)dig;
        else x[r - 8].im = (double)dig;
    }
}

// one CMux step of wave q (w = c = q >> 1, d = h = q & 1)
__device__ __forceinline__ void cmux_v9(V9Shared &sh, const V9Args &g, const V9Tw &tw, const Tw4 &tA, int i, int a,
                                        int q, int L, uint32_t (&acc)[16], double &mx, uint32_t &hlo,
                                        uint32_t &hhi, uint32_t &bad) {
    const int w = q >> 1, d = q & 1;
    double2 *X = sh.S[q];
    // 1. rotation + digit d of (X^a - 1) ACC_w, folded z_n = v_n + i v_{n+512} (layout A)
    Cx x[1][8];
    rotate_digit(acc, a, d, L, x[0]);
    // 2. forward transform of that digit polynomial (passes A, B in this wave's buffer)
    fft_fwd_AB_t<1>(x, X, tA, tw.fB, L);
    // the key rows of this wave's output / half: 16 loads in flight during pass C and the barrier
    Cx kv[4][4];
    {
        const double2 *kp = g.bk9 + ((((size_t)i * 2 + w) * 2 + d) * 16) * 64 + L;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < 4; ++t) kv[r][t] = ld_key(kp + (r * 4 + t) * 64);
    }
    __builtin_amdgcn_sched_barrier(0);
    fft_fwd_C<1>(x, tw.fC);
    store_C(X, x[0], L);                // spectrum of TGSW row 2w + d, slot 8 L + r
    lds_barrier6();                     // B2: all four spectra in LDS
    // 3. MAC over half h of output c = w: slots 256 h + 4 L + t of the four spectra
    Cx y[4];
    {
        const int s0 = 256 * d + 4 * L;
        const int off = 9 * (s0 >> 3) + (s0 & 7);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            Cx sp[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) sp[t] = ld(sh.S[r] + off + t);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const Cx &b = kv[r][t];
                if (r == 0) {
                    y[t].re = sp[t].re * b.re;
                    y[t].im = sp[t].re * b.im;
                } else {
                    y[t].re = fma_(sp[t].re, b.re, y[t].re);
                    y[t].im = fma_(sp[t].re, b.im, y[t].im);
                }
                y[t].re = fma_(-sp[t].im, b.im, y[t].re);
                y[t].im = fma_(sp[t].im, b.re, y[t].im);
            }
        }
    }
    // 4. DIT stages 0..7 of the half (256 points, 4 per lane)
    double2 *T = sh.T[q];
    pass4_first(y);
    transpose4<lay_P, lay_Q>(T, y, L);
    pass4(y, tw.w2, tw.w3);
    transpose4<lay_Q, lay_R>(T, y, L);
    pass4(y, tw.w4, tw.w5);
    transpose4<lay_R, lay_S>(T, y, L);
    pass4(y, tw.w6, tw.w7);
    // 5. stage-8 exchange: h = 0 sends zeta^-L U0, h = 1 sends W_8(L + 64 t) zeta^-L U1
    //    (W_8(L + 64 t) = W_8(L) e^{-i pi t / 4})
    {
        constexpr double hh = 0.70710678118654752440;
        y[0] = cmul(y[0], tw.sc);
        y[1] = cmul(y[1], d ? cmul(tw.sc, Cx{hh, -hh}) : tw.sc);
        y[2] = cmul(y[2], d ? Cx{tw.sc.im, -tw.sc.re} : tw.sc);
        y[3] = cmul(y[3], d ? cmul(tw.sc, Cx{-hh, -hh}) : tw.sc);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) st(T + lay_S(L, t), y[t]);
    lds_barrier6();                     // B3: both halves of both outputs in LDS
    Cx o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = ld(sh.T[q ^ 1] + lay_S(L, t));
    // 6. stage 8 (twiddle folded into the sent half), register post-twist e^{-2 pi i r / 32}, rint
    Cx X8[8];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const Cx &u0 = d ? o[t] : y[t];
        const Cx &v1 = d ? y[t] : o[t];
        X8[t] = Cx{u0.re + v1.re, u0.im + v1.im};
        X8[t + 4] = Cx{u0.re - v1.re, u0.im - v1.im};
    }
    constexpr double kOm[8][2] = {
        {1.0, 0.0},
        {0.98078528040323044913, -0.19509032201612826785},
        {0.92387953251128675613, -0.38268343236508977173},
        {0.83146961230254523708, -0.55557023301960222474},
        {0.70710678118654752440, -0.70710678118654752440},
        {0.55557023301960222474, -0.83146961230254523708},
        {0.38268343236508977173, -0.92387953251128675613},
        {0.19509032201612826785, -0.98078528040323044913}};
#pragma unroll
    for (int r = 1; r < 8; ++r) X8[r] = cmul(X8[r], Cx{kOm[r][0], kOm[r][1]});
    // acc_c += rint(result): coefficient L + 64 r (re) and L + 64 (r + 8) (im); the 1/8 rule
    // through the quarter-ulp shifter (fft_wave.h torus_of_qchk), the distance sampled once
    mx = __builtin_fmax(mx, __builtin_fabs(X8[0].re - __builtin_rint(X8[0].re)));
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        acc[r] += torus_of_qchk(X8[r].re, bad, hlo, hhi);
        acc[r + 8] += torus_of_qchk(X8[r].im, bad, hlo, hhi);
    }
}

__device__ __forceinline__ V9Tw load_tw9(const V9Args &g, int d, int L) {
    V9Tw t;
    t.fB = load_tw(g.tw, 0, L);
    t.fC = load_tw(g.tw, 1, L);
    const double2 *p = g.tw9 + L;
    t.w2 = ld(p);
    t.w3 = ld(p + 64);
    t.w4 = ld(p + 128);
    t.w5 = ld(p + 192);
    t.w6 = ld(p + 256);
    t.w7 = ld(p + 320);
    t.sc = ld(p + (d ? 448 : 384));
    return t;
}

// prologue (gate / row linear combination + modulus switching), 500 CMux steps, extraction
__device__ __forceinline__ void br_v9_body(V9Shared &sh, const V9Args &g, const RowTerms6 &t, int32_t mu,
                                           int32_t *__restrict__ ua, int32_t *__restrict__ ub, size_t slot) {
    const int tid = threadIdx.x;
    const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = tid & 63;
    const int w = q >> 1, d = q & 1;
    // gate prologue + modulus switching (lwe-bootstrapping-functions-fft.cu:1851-1858)
    for (int i = tid; i < kn; i += kV9Threads) {
        uint32_t x = t.xa ? (uint32_t)t.sa * (uint32_t)t.xa[i] : 0u;
        if (t.ya) x += (uint32_t)t.sb * (uint32_t)t.ya[i];
        if (t.za) x += (uint32_t)t.sc * (uint32_t)t.za[i];
        sh.bara[i] = (short)modswitch_2N(x);
    }
    if (tid == 0) {
        uint32_t xb = (uint32_t)t.c + (t.xb ? (uint32_t)t.sa * (uint32_t)t.xb[0] : 0u);
        if (t.yb) xb += (uint32_t)t.sb * (uint32_t)t.yb[0];
        if (t.zb) xb += (uint32_t)t.sc * (uint32_t)t.zb[0];
        sh.barb = modswitch_2N(xb);
    }
    const V9Tw tw = load_tw9(g, d, L);
    const Tw4 tA = load_tw_sgpr(g.tw);
    __syncthreads();
    // ACC = (0, X^{2N - barb} (mu, ..., mu)) (:1427-1431); both waves of a pair hold polynomial w
    uint32_t acc[16];
    {
        const int e = (k2N - sh.barb) & (k2N - 1);
#pragma unroll
        for (int r = 0; r < 16; ++r)
            acc[r] = w == 0 ? 0u : (((L + 64 * r - e) & (k2N - 1)) < kN ? (uint32_t)mu : 0u - (uint32_t)mu);
    }
    double mx = 0.0;
    uint32_t hlo = kQShiftHiLo, hhi = kQShiftHiLo, bad = 0;
    int a_next = sh.bara[0];
    for (int i = 0; i < kn; ++i) {
        const int a = a_next;
        a_next = sh.bara[i + 1 < kn ? i + 1 : i];
        if (a == 0) continue;   // X^0 - 1 = 0: identity CMux (:705); uniform over the workgroup
        cmux_v9(sh, g, tw, tA, i, a, q, L, acc, mx, hlo, hhi, bad);
    }
    if (g.flags && d == 0) {   // exactness guard: output w's largest rounding distance (high word)
        if (bad || hlo < kQShiftHiLo || hhi >= kQShiftHiEnd) mx = 0.5;
        const uint32_t h = wave_max_hi(mx);
        if (L == 0) {
            g.flags[2 * slot + w] = h;
            atomicMax(g.stats + 1, h);
        }
    }
    // sample extraction at index 0 (lwe.cu:41-56): a_j = -acc_a[N - j] = E_a[2N - j]
    __syncthreads();
    if (q == 0) {
        uint32_t *E = reinterpret_cast<uint32_t *>(sh.S[0]);
        write_ext(E, acc, L);
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int j = L + 64 * r;
            ua[j] = (int32_t)E[(k2N - j) & (k2N - 1)];
        }
    } else if (q == 2 && L == 0) {
        *ub = (int32_t)acc[0];
    }
}

__global__ __launch_bounds__(kV9Threads, 2) void k_blind_rotate_v9(V9Args g, int B, int base, BrInput in0, BrInput in1,
                                                                   int32_t mu, int32_t *__restrict__ u_a,
                                                                   int32_t *__restrict__ u_b) {
    __shared__ V9Shared sh;
    const int gct = base + blockIdx.x;
    const int half = gct >= B;
    const int idx = half ? gct - B : gct;
    const BrInput &in = half ? in1 : in0;
    RowTerms6 t;
    t.c = in.c; t.sa = in.sa; t.sb = in.sb; t.sc = 0;
    t.xa = in.x_a + (size_t)idx * kn; t.xb = in.x_b + idx;
    t.ya = in.sb ? in.y_a + (size_t)idx * kn : nullptr; t.yb = in.sb ? in.y_b + idx : nullptr;
    t.za = nullptr; t.zb = nullptr;
    br_v9_body(sh, g, t, mu, u_a + (size_t)gct * kN, u_b + gct, (size_t)gct);
}

__global__ __launch_bounds__(kV9Threads, 2) void k_blind_rotate_v9_rows(V9Args g, int B, long base,
                                                                        const CircRow *__restrict__ rows,
                                                                        const int32_t *__restrict__ wa,
                                                                        const int32_t *__restrict__ wb, int32_t mu,
                                                                        int32_t *__restrict__ u_a,
                                                                        int32_t *__restrict__ u_b) {
    __shared__ V9Shared sh;
    const long flat = base + blockIdx.x;          // row-major (row, instance)
    const int r = (int)(flat / B), k = (int)(flat - (long)r * B);
    const CircRow row = rows[r];
    auto wire = [&](int wi, const int32_t *&pa, const int32_t *&pb) {
        if (wi < 0) { pa = nullptr; pb = nullptr; return; }
        const size_t s = (size_t)wi * B + k;
        pa = wa + s * kn;
        pb = wb + s;
    };
    RowTerms6 t;
    t.c = row.c; t.sa = row.sa; t.sb = row.sb; t.sc = row.sc;
    wire(row.x, t.xa, t.xb);
    wire(row.y, t.ya, t.yb);
    wire(row.z, t.za, t.zb);
    const size_t slot = (size_t)r * B + k;
    br_v9_body(sh, g, t, mu, u_a + slot * kN, u_b + slot, slot);
}

// raw CMux steps on explicit accumulators acc [B][2][kN] (debug / parity entry, unguarded)
__global__ __launch_bounds__(kV9Threads, 2) void k_blind_rotate_v9_debug(V9Args g, int iters, int32_t *__restrict__ acc,
                                                                         const int32_t *__restrict__ bara) {
    __shared__ V9Shared sh;
    const int tid = threadIdx.x;
    const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = tid & 63;
    const int w = q >> 1, d = q & 1;
    int32_t *accg = acc + (size_t)blockIdx.x * 2 * kN + (size_t)w * kN;
    uint32_t ac[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) ac[r] = (uint32_t)accg[L + 64 * r];
    for (int i = tid; i < iters; i += kV9Threads) sh.bara[i] = (short)(bara[(size_t)blockIdx.x * iters + i] & (k2N - 1));
    const V9Tw tw = load_tw9(g, d, L);
    const Tw4 tA = load_tw_sgpr(g.tw);
    __syncthreads();
    double mx = 0.0;
    uint32_t hlo = kQShiftHiLo, hhi = kQShiftHiLo, bad = 0;
    for (int i = 0; i < iters; ++i) {
        const int a = sh.bara[i];
        if (a == 0) continue;
        cmux_v9(sh, g, tw, tA, i, a, q, L, ac, mx, hlo, hhi, bad);
    }
    __syncthreads();
    if (d == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) accg[L + 64 * r] = (int32_t)ac[r];
    }
}

// the FFT-domain key re-laid per (output c, half h): bk9[i][c][h][row][t][L] = slot 256 h + 4 L + t
// of bk_fft[i][row][c] (slot 8 L' + r' at [r'][L'])
__global__ __launch_bounds__(256) void k_bk_fft_to_v9(const double2 *__restrict__ bkf, double2 *__restrict__ bk9) {
    const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;   // destination element
    const size_t total = (size_t)kn * 2 * 2 * 4 * 4 * 64;
    if (e >= total) return;
    const int L = (int)(e & 63), t = (int)((e >> 6) & 3), row = (int)((e >> 8) & 3), h = (int)((e >> 10) & 1),
              c = (int)((e >> 11) & 1);
    const size_t i = e >> 12;
    const int s = 256 * h + 4 * L + t;
    bk9[e] = bkf[((i * 4 + row) * 2 + c) * 512 + (size_t)(s & 7) * 64 + (s >> 3)];
}

}  // namespace

// inverse-stage and post-twist lane tables of the v9 kernel (double2 [8][64]): W_2(L & 3),
// W_3(L & 3), W_4(L & 15), W_5(L & 15), W_6(L), W_7(L), zeta^-L, W_8(L) zeta^-L, where
// W_k(j) = e^{-i pi j / 2^k} (scripts/emu_v9.py)
void build_v9_twiddles(double2 *tw) {
    const long double pi = 3.14159265358979323846264338327950288L;
    auto W = [&](int k, int j) {
        const long double th = -pi * (long double)j / (long double)(1 << k);
        return make_double2((double)cosl(th), (double)sinl(th));
    };
    auto zeta = [&](int L) {   // e^{-i pi L / 1024}
        const long double th = -pi * (long double)L / 1024.0L;
        return make_double2((double)cosl(th), (double)sinl(th));
    };
    for (int L = 0; L < 64; ++L) {
        tw[0 * 64 + L] = W(2, L & 3);
        tw[1 * 64 + L] = W(3, L & 3);
        tw[2 * 64 + L] = W(4, L & 15);
        tw[3 * 64 + L] = W(5, L & 15);
        tw[4 * 64 + L] = W(6, L);
        tw[5 * 64 + L] = W(7, L);
        tw[6 * 64 + L] = zeta(L);
        const long double th = -pi * (long double)L / 256.0L - pi * (long double)L / 1024.0L;
        tw[7 * 64 + L] = make_double2((double)cosl(th), (double)sinl(th));
    }
}

hipError_t launch_bk_fft_to_v9(const double2 *d_bkf, double2 *d_bk9, hipStream_t s) {
    const size_t total = (size_t)kn * 2 * 2 * 4 * 4 * 64;
    hipLaunchKernelGGL(k_bk_fft_to_v9, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, d_bkf, d_bk9);
    return hipGetLastError();
}

static V9Args v9_args(const DeviceKey &key, const Guard *guard) {
    V9Args g;
    g.bk9 = key.bk9;
    g.tw = key.tw6;
    g.tw9 = key.tw9;
    g.flags = guard ? guard->flags : nullptr;
    g.stats = guard ? guard->stats : nullptr;
    return g;
}

hipError_t launch_blind_rotate_v9(const DeviceKey &key, int B, int halves, const BrInput *in, int32_t mu,
                                  int32_t *u_a, int32_t *u_b, hipStream_t s, const Guard *guard) {
    if (B <= 0) return hipSuccess;
    if (!key.bk9 || !key.tw9) return hipErrorInvalidValue;
    const BrInput in1 = halves > 1 ? in[1] : in[0];
    const long total = (long)B * halves;
    if (total > 0x7fffffffL) return hipErrorInvalidValue;
    trace_kernel("k_blind_rotate_v9(4-wave)");
    hipLaunchKernelGGL(k_blind_rotate_v9, dim3((unsigned)total), dim3(kV9Threads), 0, s, v9_args(key, guard), B, 0,
                       in[0], in1, mu, u_a, u_b);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_v9_rows(const DeviceKey &key, int B, int nrows, const CircRow *rows, const int32_t *wa,
                                       const int32_t *wb, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t s,
                                       const Guard *guard) {
    if (B <= 0 || nrows <= 0) return hipSuccess;
    if (!key.bk9 || !key.tw9) return hipErrorInvalidValue;
    const long total = (long)B * nrows;
    if (total > 0x7fffffffL) return hipErrorInvalidValue;
    trace_kernel("k_blind_rotate_v9_rows(4-wave)");
    hipLaunchKernelGGL(k_blind_rotate_v9_rows, dim3((unsigned)total), dim3(kV9Threads), 0, s, v9_args(key, guard), B,
                       0L, rows, wa, wb, mu, u_a, u_b);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_v9_debug(const DeviceKey &key, int B, int iters, int32_t *acc, const int32_t *bara,
                                        hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (iters < 0 || iters > kn || !key.bk9 || !key.tw9) return hipErrorInvalidValue;
    trace_kernel("k_blind_rotate_v9_debug(4-wave)");
    hipLaunchKernelGGL(k_blind_rotate_v9_debug, dim3(B), dim3(kV9Threads), 0, s, v9_args(key, nullptr), iters, acc,
                       bara);
    return hipGetLastError();
}

}  // namespace tfhe_amd
