// blind_rotate_v12.hip — the latency-regime blind rotation: four waves per ciphertext, each with
// two independent half-transform chains (data flow emulated in scripts/emu_v12.py).
//
// tfhe_blindRotate_FFT (lwe-bootstrapping-functions-fft.cu:676-737) with the external product of
// tGswFFTExternMulToTLwe (tgsw-fft-operations.cu:124-264) in v6's fp64 arithmetic (the same
// spectrum, slot for slot, the same key, the same rounding and exactness guard), re-partitioned for
// launches of at most one ciphertext per CU.  There v6 runs two waves on two of the CU's four SIMDs
// and each wave's own VALU issue (~1 040 instructions per CMux step, a lone wave issuing one fp64
// instruction per ~7 cycles) is ~85 % of the step.  v12 uses all four SIMDs:
//
//  * the 512-point transform splits at its first Cooley-Tukey stage: stage 0 maps (z_n, z_{n+256})
//    to u + W0 v (slots 0..255, half 0) and u - W0 v (half 1), and every later stage stays inside
//    one half.  Wave (w, h) holds the whole accumulator polynomial w (the same 16 Torus32 per lane
//    in both waves of the pair), computes all of its digits, only its half of stage 0, then stages
//    1..8 of that half for BOTH digit polynomials: two independent chains, 4 complex per lane
//    each, four radix-4 passes (layouts A' B' C' D', three LDS transposes, conflict-free slot maps);
//  * MAC of its half of the slots with BK_i (v6's key layout, buffer loads), the partial sum of
//    output 1 - w handed to wave (1 - w, h) through LDS (barrier 1), the partner's partial seeding
//    the MAC of output w;
//  * the DIT inverse of output w inside its half (stages 0..7; the post-twist's lane factor folded
//    into pass A'), the half handed to wave (w, 1 - h) (barrier 2), then stage 8, the register
//    factors of the post-twist and the rounding (v6's quarter-ulp guard) of all 16 coefficients in
//    both waves, so that both hold the new accumulator.
// Per wave and step: ~500 fp64 (v6: 851) and ~170 other VALU instructions, two barriers.
#include <atomic>
#include "engine.h"
#include "modarith.h"
#include "fft_wave.h"

namespace tfhe_amd {

namespace {

constexpr int kV12Threads = 256;
constexpr int kTBStride = 320;                   // one polynomial's transpose slots (256 + the C <-> D pad)

struct __attribute__((aligned(16))) V12Shared {
    double2 TB[4][2 * kTBStride];                // per wave: the forward's two polynomials / the inverse's one
    double2 HB[4][kTBStride];                    // per wave: the partial sum handed over (layout D')
    double2 XB[4][256];                          // per wave: the inverse's half handed over (layout A')
    short bara[512];
    int barb;
};

// positions m (0..255) inside a half, lane L, register r < 4
__device__ __forceinline__ int mA(int L, int r) { return L + 64 * r; }
__device__ __forceinline__ int mB(int L, int r) { return (L & 15) + 16 * r + 64 * (L >> 4); }
__device__ __forceinline__ int mC(int L, int r) { return (L & 3) + 4 * r + 16 * (L >> 2); }
__device__ __forceinline__ int mD(int L, int r) { return 4 * L + r; }
// LDS slot maps, conflict-free for the 16-B stores (8-lane groups, 128-B rows) and loads (16-lane
// groups, 256-B rows) of every transpose they serve (searched exhaustively over simple families)
__device__ __forceinline__ int sAB(int m) { return m; }                                  // A' <-> B'
__device__ __forceinline__ int sBC(int m) { return m ^ (((m >> 4) & 3) << 2); }          // B' <-> C'
__device__ __forceinline__ int sCD(int m) { return m + (m >> 2); }                       // C' <-> D', hand-off

// per-lane twiddles, loop-invariant, in registers: the forward's passes B', C', D' (stage a, stage
// b; the odd pair of stage b takes i x it) and the inverse's passes C', B', A', stage 8, zeta^-L
struct Tw12 {
    Cx f[6];
    Cx i8, i16, i32, i64, i128s, i256, sig, c512, c512b;
};
// the global table (build_v6_twiddles, kTw12): [h][6][64] forward, then [9][64] inverse
__device__ __forceinline__ Tw12 load_tw12(const double2 *tw, int h, int L) {
    Tw12 t;
    const double2 *f = tw + kTw12 + h * 6 * 64 + L;
#pragma unroll
    for (int k = 0; k < 6; ++k) t.f[k] = ld(f + 64 * k);
    const double2 *q = tw + kTw12 + 12 * 64 + L;
    t.i8 = ld(q);
    t.i16 = ld(q + 64);
    t.i32 = ld(q + 128);
    t.i64 = ld(q + 192);
    t.i128s = ld(q + 256);
    t.i256 = ld(q + 320);
    t.sig = ld(q + 384);
    t.c512 = ld(q + 448);
    t.c512b = ld(q + 512);
    return t;
}

// radix-4 forward pass: stage a at register distance 2 (ta), stage b at distance 1 (tb; i tb for
// the pair (2, 3))
__device__ __forceinline__ void fwd4(Cx (&x)[4], const Cx &ta, const Cx &tb) {
    bf_fwd<false>(x[0], x[2], ta);
    bf_fwd<false>(x[1], x[3], ta);
    bf_fwd<false>(x[0], x[1], tb);
    bf_fwd<true>(x[2], x[3], tb);
}
// radix-2 DIT stages at register distance 1 (a) and 2 (b for (0, 2), -i b for (1, 3))
__device__ __forceinline__ void dit4(Cx (&x)[4], const Cx &a, const Cx &b) {
    bf_fwd<false>(x[0], x[1], a);
    bf_fwd<false>(x[2], x[3], a);
    bf_fwd<false>(x[0], x[2], b);
    bf_fwd<true>(x[1], x[3], negi_(b));
}
// u + W v only (one output of a butterfly): 4 FMAs
__device__ __forceinline__ Cx half_bf(const Cx &u, const Cx &v, const Cx &w) {
    return Cx{fma_(-w.im, v.im, fma_(w.re, v.re, u.re)), fma_(w.im, v.re, fma_(w.re, v.im, u.im))};
}

template <int NP, class FS, class FL>
__device__ __forceinline__ void transpose12(Cx (&x)[NP][4], double2 *buf, int L, FS slot_st, FL slot_ld) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int r = 0; r < 4; ++r) st(buf + p * kTBStride + slot_st(L, r), x[p][r]);
    wave_sync();
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int r = 0; r < 4; ++r) x[p][r] = ld(buf + p * kTBStride + slot_ld(L, r));
    wave_sync();
}

struct V12Args {
    const double2 *bk;   // v6's FFT-domain key / 512: [kn][4 rows][2 c][8 r6][64 L6], slot 8 L6 + r6
    uint32_t *flags;     // exactness guard (engine.h Guard), or null
    uint32_t *stats;
    const double2 *tw;   // build_v6_twiddles' table
};

// one CMux step of wave (w, H): acc += [(X^a - 1) ACC] (x) BK_i, this wave's copy of polynomial w
template <int H>
__device__ __forceinline__ void cmux_v12(V12Shared &sh, const V12Args &g, __amdgpu_buffer_rsrc_t rk, const Tw4 &tu,
                                         const Tw12 &t, int i, int a, int w, int wv, int L, int kvoff,
                                         uint32_t (&acc)[16], double &mx, uint32_t &hlo, uint32_t &hhi,
                                         uint32_t &bad) {
    // X^a ACC_w in registers (cmux_v6's RREG rotation: ds_bpermute by s = a mod 64, then the
    // negacyclic register rotation by q = a / 64 in five conditional stages), then the signed
    // gadget digits (tgsw-functions.cu:322-351) of (X^a - 1) ACC_w, folded z_n = d_n + i d_{n+512}
    Cx D[2][8];
    {
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
                uint32_t tt[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) tt[r] = r >= K ? V[r - K] : 0u - V[r + 16 - K];
#pragma unroll
                for (int r = 0; r < 16; ++r) V[r] = tt[r];
            }
        }
        const bool lo = L < s;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t rot = lo ? (r ? V[r - 1] : 0u - V[15]) : V[r];
            const uint32_t diff = rot - acc[r];
            const int32_t hi = (int32_t)(diff + (kDecompOffset + 0x80000000u)) >> 22;
            const int32_t lw = __builtin_amdgcn_sbfe((int32_t)(diff + (kDecompOffset + 0x200000u)), 12, 10);
            if (r < 8) {
                D[0][r].re = (double)hi;
                D[1][r].re = (double)lw;
            } else {
                D[0][r - 8].im = (double)hi;
                D[1][r - 8].im = (double)lw;
            }
        }
    }
    // the key slices of this half for both outputs: slot n = 256 H + 4 L + r lies at v6's [r6][L6] =
    // [4 (L & 1) + r][32 H + (L >> 1)]; rows 2w + p, output c: soffset (i 8 + 4 w + 2 p + c) x 8 KB
    Cx kb[2][2][4];   // [first (output 1 - w) / second (output w)][p][r]: static indices only (no scratch)
    auto load_keys = [&]() {
        const int row0 = i * 8 + w * 4;
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int c = k == 0 ? 1 - w : w;
                const int so = __builtin_amdgcn_readfirstlane((row0 + 2 * p + c) * 512 * 16);
#pragma unroll
                for (int r = 0; r < 4; ++r) kb[k][p][r] = ld_key_buf(rk, kvoff + r * 1024, so);
            }
        __builtin_amdgcn_sched_barrier(0);
    };
#ifndef V12_KEY_AT
#define V12_KEY_AT 2   // measured best: 0 +8.6 %, 1 +1.4 %, 3 +1.6 % at B = 1
#endif
    if (V12_KEY_AT == 3) load_keys();
    // forward: this half of stage 0 (w0 negated for half 1), then pass A' (stages 1, 2: uniform
    // twiddles W[1][H], W[2][2H])
    Cx x[2][4];
    {
        const Cx w0 = H ? Cx{-tu.w0.re, -tu.w0.im} : tu.w0;
        const Cx w1 = H ? Cx{-tu.w1.im, tu.w1.re} : tu.w1;          // W[1][1] = i W[1][0]
        const Cx &w2 = H ? tu.w2b : tu.w2a;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
#pragma unroll
            for (int r = 0; r < 4; ++r) x[p][r] = half_bf(D[p][r], D[p][r + 4], w0);
            fwd4(x[p], w1, w2);
        }
    }
    double2 *T = sh.TB[wv];
    transpose12<2>(x, T, L, [](int l, int r) { return sAB(mA(l, r)); }, [](int l, int r) { return sAB(mB(l, r)); });
    if (V12_KEY_AT == 2) load_keys();
#pragma unroll
    for (int p = 0; p < 2; ++p) fwd4(x[p], t.f[0], t.f[1]);
    transpose12<2>(x, T, L, [](int l, int r) { return sBC(mB(l, r)); }, [](int l, int r) { return sBC(mC(l, r)); });
    if (V12_KEY_AT == 1) load_keys();
#pragma unroll
    for (int p = 0; p < 2; ++p) fwd4(x[p], t.f[2], t.f[3]);
    transpose12<2>(x, T, L, [](int l, int r) { return sCD(mC(l, r)); }, [](int l, int r) { return sCD(mD(l, r)); });
    if (V12_KEY_AT == 0) load_keys();
#pragma unroll
    for (int p = 0; p < 2; ++p) fwd4(x[p], t.f[4], t.f[5]);
    // MAC: output 1 - w first, handed to wave (1 - w, H); then output w seeded with the partner's
    Cx Y[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const Cx &k0 = kb[0][0][r], &k1 = kb[0][1][r];
        double re = x[0][r].re * k0.re, im = x[0][r].re * k0.im;
        re = fma_(-x[0][r].im, k0.im, re);
        im = fma_(x[0][r].im, k0.re, im);
        re = fma_(x[1][r].re, k1.re, re);
        im = fma_(x[1][r].re, k1.im, im);
        re = fma_(-x[1][r].im, k1.im, re);
        im = fma_(x[1][r].im, k1.re, im);
        Y[r] = Cx{re, im};
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) st(sh.HB[wv] + sCD(mD(L, r)), Y[r]);
    lds_barrier6();                                     // barrier 1: partial sums handed over
    {
        Cx o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = ld(sh.HB[wv ^ 1] + sCD(mD(L, r)));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const Cx &k0 = kb[1][0][r], &k1 = kb[1][1][r];
            double re = fma_(x[0][r].re, k0.re, o[r].re), im = fma_(x[0][r].re, k0.im, o[r].im);
            re = fma_(-x[0][r].im, k0.im, re);
            im = fma_(x[0][r].im, k0.re, im);
            re = fma_(x[1][r].re, k1.re, re);
            im = fma_(x[1][r].re, k1.im, im);
            re = fma_(-x[1][r].im, k1.im, re);
            im = fma_(x[1][r].im, k1.re, im);
            Y[r] = Cx{re, im};
        }
    }
    // inverse of output w inside this half: D' stages 0, 1 (twiddles 1, -i), C' 2, 3, B' 4, 5, A' 6, 7
    bf_one(Y[0], Y[1]);
    bf_one(Y[2], Y[3]);
    bf_one(Y[0], Y[2]);
    bf_negi(Y[1], Y[3]);
    {
        Cx y1[1][4] = {{Y[0], Y[1], Y[2], Y[3]}};
        transpose12<1>(y1, T, L, [](int l, int r) { return sCD(mD(l, r)); }, [](int l, int r) { return sCD(mC(l, r)); });
        dit4(y1[0], t.i8, t.i16);
        transpose12<1>(y1, T, L, [](int l, int r) { return sBC(mC(l, r)); }, [](int l, int r) { return sBC(mB(l, r)); });
        dit4(y1[0], t.i32, t.i64);
        transpose12<1>(y1, T, L, [](int l, int r) { return sAB(mB(l, r)); }, [](int l, int r) { return sAB(mA(l, r)); });
        y1[0][0] = cmul(y1[0][0], t.sig);
        y1[0][2] = cmul(y1[0][2], t.sig);
        dit4(y1[0], t.i128s, t.i256);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            Y[r] = y1[0][r];
            st(sh.XB[wv] + mA(L, r), Y[r]);
        }
    }
    lds_barrier6();                                     // barrier 2: halves handed over
    Cx z[8];
    {
        Cx o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = ld(sh.XB[wv ^ 2] + mA(L, r));
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            z[4 * H + r] = Y[r];
            z[4 * (1 - H) + r] = o[r];
        }
    }
    // stage 8 across the halves, the post-twist's register factors e^{-2 pi i r / 32}
    bf_fwd<false>(z[0], z[4], t.c512);
    bf_fwd<false>(z[1], z[5], t.c512b);
    bf_fwd<true>(z[2], z[6], negi_(t.c512));
    bf_fwd<true>(z[3], z[7], negi_(t.c512b));
    {
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
        for (int r = 1; r < 8; ++r) z[r] = cmul(z[r], Cx{kOm[r][0], kOm[r][1]});
    }
    // acc_w += rint(result) with the exactness guard (cmux_v6's rounding)
    mx = __builtin_fmax(mx, __builtin_fabs(z[0].re - __builtin_rint(z[0].re)));
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        acc[r] += torus_of_qchk(z[r].re, bad, hlo, hhi);
        acc[r + 8] += torus_of_qchk(z[r].im, bad, hlo, hhi);
    }
}

template <int H>
__device__ __forceinline__ void br_v12_loop(V12Shared &sh, const V12Args &g, const Tw4 &tu, int w, int wv, int L,
                                            uint32_t (&acc)[16], double &mx, uint32_t &hlo, uint32_t &hhi,
                                            uint32_t &bad) {
    const Tw12 t = load_tw12(g.tw, H, L);
    const __amdgpu_buffer_rsrc_t rk = key_rsrc(g.bk);
    const int kvoff = (256 * (L & 1) + 32 * H + (L >> 1)) * 16;
    int a_next = sh.bara[0];
    for (int i = 0; i < kn; ++i) {
        const int a = a_next;
        a_next = sh.bara[i + 1 < kn ? i + 1 : i];
        if (a == 0) continue;   // X^0 - 1 = 0: identity CMux (:705), all four waves alike
        cmux_v12<H>(sh, g, rk, tu, t, i, a, w, wv, L, kvoff, acc, mx, hlo, hhi, bad);
    }
}

__global__ __launch_bounds__(kV12Threads, 1) void k_blind_rotate_v12(V12Args g, int B, int base, BrInput in0,
                                                                     BrInput in1, int32_t mu,
                                                                     int32_t *__restrict__ u_a,
                                                                     int32_t *__restrict__ u_b) {
    __shared__ V12Shared sh;
    const int gct = base + blockIdx.x;
    const int half = gct >= B;
    const int idx = half ? gct - B : gct;
    const BrInput &in = half ? in1 : in0;
    const int tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wv & 1, h = wv >> 1;
    const int L = tid & 63;
    // gate prologue + modulus switching (lwe-bootstrapping-functions-fft.cu:1851-1858)
    const int32_t *xa = in.x_a + (size_t)idx * kn, *ya = in.sb ? in.y_a + (size_t)idx * kn : nullptr;
    for (int j = tid; j < kn; j += kV12Threads) {
        uint32_t x = (uint32_t)in.sa * (uint32_t)xa[j];
        if (ya) x += (uint32_t)in.sb * (uint32_t)ya[j];
        sh.bara[j] = (short)modswitch_2N(x);
    }
    if (tid == 0) {
        uint32_t xb = (uint32_t)in.c + (uint32_t)in.sa * (uint32_t)in.x_b[idx];
        if (in.sb) xb += (uint32_t)in.sb * (uint32_t)in.y_b[idx];
        sh.barb = modswitch_2N(xb);
    }
    const Tw4 tu = load_tw_sgpr(g.tw);
    __syncthreads();
    // ACC = (0, X^{2N - barb} (mu, ..., mu)) (:1427-1431), in both waves of the pair
    uint32_t acc[16];
    {
        const int e = (k2N - sh.barb) & (k2N - 1);
#pragma unroll
        for (int r = 0; r < 16; ++r)
            acc[r] = w == 0 ? 0u : (((L + 64 * r - e) & (k2N - 1)) < kN ? (uint32_t)mu : 0u - (uint32_t)mu);
    }
    double mx = 0.0;
    uint32_t hlo = kQShiftHiLo, hhi = kQShiftHiLo, bad = 0;
    if (h == 0) br_v12_loop<0>(sh, g, tu, w, wv, L, acc, mx, hlo, hhi, bad);
    else br_v12_loop<1>(sh, g, tu, w, wv, L, acc, mx, hlo, hhi, bad);
    const size_t slot = (size_t)gct;
    if (g.flags && h == 0) {   // exactness guard: both waves of the pair computed the same roundings
        if (bad || hlo < kQShiftHiLo || hhi >= kQShiftHiEnd) mx = 0.5;
        const uint32_t hw = wave_max_hi(mx);
        if (L == 0) {
            g.flags[2 * slot + w] = hw;
            atomicMax(g.stats + 1, hw);
        }
    }
    // sample extraction at index 0 (lwe.cu:41-56): a_j = -acc_a[N - j] = E_a[2N - j]
    __syncthreads();
    if (wv == 0) {
        uint32_t *E = reinterpret_cast<uint32_t *>(sh.TB[0]);
        write_ext(E, acc, L);
        wave_sync();
        int32_t *ua = u_a + (size_t)gct * kN;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int j = L + 64 * r;
            ua[j] = (int32_t)E[(k2N - j) & (k2N - 1)];
        }
    } else if (wv == 1 && L == 0) {
        u_b[gct] = (int32_t)acc[0];
    }
}
static_assert(kExt6 * 4 <= 2 * kTBStride * 16, "the extraction's extension fits a wave's transpose buffer");

}  // namespace

// v12 for launches of at most one ciphertext per CU
hipError_t launch_blind_rotate_v12(const DeviceKey &key, int B, int halves, const BrInput *in, int32_t mu,
                                   int32_t *u_a, int32_t *u_b, hipStream_t s, const Guard *guard, long base,
                                   long n) {
    const BrInput in1 = halves > 1 ? in[1] : in[0];
    V12Args g;
    g.bk = key.bk_fft;
    g.flags = guard ? guard->flags : nullptr;
    g.stats = guard ? guard->stats : nullptr;
    g.tw = key.tw6;
    trace_kernel("k_blind_rotate_v12(four-wave)");
    hipLaunchKernelGGL(k_blind_rotate_v12, dim3((unsigned)n), dim3(kV12Threads), 0, s, g, B, (int)base, in[0], in1,
                       mu, u_a, u_b);
    return hipGetLastError();
}

}  // namespace tfhe_amd
