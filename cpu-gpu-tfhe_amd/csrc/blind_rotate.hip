// blind_rotate.hip — v2 blind rotation for gfx950: register-resident exact NTTs.
//
// Same contract as bootstrap.hip's v1 (tfhe_blindRotate_FFT + extraction,
// lwe-bootstrapping-functions-fft.cu:676-737, 1408-1456, 1834-1870; tGswFFTExternMulToTLwe
// tgsw-fft-operations.cu:124-264), re-laid out for CDNA4:
//
//  * one 128-thread workgroup (2 waves) per ciphertext; wave s owns prime q_s.  It holds the
//    4 digit polynomials of the decomposed accumulator (4 x 16 values per lane) through the
//    forward NTT, the pointwise MAC with BK_i and the 2 inverse NTTs in VGPRs;
//  * a 1024-point negacyclic NTT = 10 radix-2 stages in 3 register layouts
//      A: lane L, reg r <-> j = L + 64 r          (stages 9..6, wave-uniform twiddles: SGPRs)
//      B: j = (L & 3) | r << 2 | (L >> 2) << 6     (stages 5..2)
//      C: j = 16 L + r                            (stages 1,0 fwd; 0..3 inv; MAC; BK loads)
//    with two LDS transposes per transform through a per-wave padded scratch
//    (word address j + 4 (j >> 6): conflict-free for b32 A/B and b128 C accesses);
//  * lazy butterflies (forward: no reductions, values < 22q since q < 2^27; inverse: Harvey [0, 2q)), Shoup
//    twiddles; lane-varying twiddles come from "stream" tables laid out in consumption
//    order (one coalesced 512-B load per slot);
//  * the MAC reads BK_i (NTT domain, Montgomery form, 1/N folded) as 16-B loads from a
//    lane-major layout, sums 4 rows in 64 bits and reduces once (REDC);
//  * the two primes meet in a CRT exchange through LDS; the accumulator lives in LDS.
#include "engine.h"
#include "modarith.h"
#include "ntt_wave.h"

#include <cstdlib>

namespace tfhe_amd {

namespace {

[[maybe_unused]] constexpr int kV2Threads = 128;
struct V2Shared {
    uint32_t acc[2][kN];               // TLWE accumulator (a, b)
    uint32_t scratch[2][kPadRow];      // one per wave (prime)
    int bara[512];
    int barb;
};

struct V2Args {
    const uint32_t *bk;   // [kn][2][2 c][4 p][4 v][64 L][4 e]   (Montgomery, 1/N folded)
    const uint2 *tu_f;    // [2][16] uniform forward twiddles (idx 1..15)
    const uint2 *tu_i;    // [2][16]
    const uint2 *ts_f;    // [2][27][64] stream forward twiddles
    const uint2 *ts_i;    // [2][18][64]
    uint32_t qinv_neg0, qinv_neg1, crt_h, crt_hp;
};

// CRT exchange + accumulate; wave S handles r in [8S, 8S+8) of both polys.  Split in a
// give (write) and a take (read + accumulate) half so that the workgroup barrier between
// them sits in uniform control flow (a barrier inside the per-wave `if (s == 0)` branches
// was miscompiled: results wrong on every coefficient).
template <int S>
__device__ __forceinline__ void crt_give(V2Shared &sh, const uint32_t (&O)[2][16], int L) {
    uint32_t *mine = sh.scratch[S];
    constexpr int give = 8 * (1 - S);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) mine[(c * 8 + rr) * 64 + L] = O[c][give + rr];
}
template <int S>
__device__ __forceinline__ void crt_take(V2Shared &sh, const uint32_t (&O)[2][16], int L, const V2Args &g) {
    const uint32_t *other = sh.scratch[1 - S];
    constexpr int keep = 8 * S;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) {
            const uint32_t xo = other[(c * 8 + rr) * 64 + L];
            const uint32_t xm = O[c][keep + rr];
            const uint32_t x0 = S == 0 ? xm : xo, x1 = S == 0 ? xo : xm;
            sh.acc[c][L + 64 * (keep + rr)] += crt_torus(x0, x1, g.crt_h, g.crt_hp);
        }
}

// one CMux step for key index i and rotation a (1..2N-1); called by both waves
__device__ __forceinline__ void cmux_v2(V2Shared &sh, const V2Args &g, int i, int a, int s, int L) {
    const uint32_t q = s ? kQ1 : kQ0;
    const uint32_t q2 = 2 * q;
    uint32_t *sc = sh.scratch[s];
    // (X^a - 1) ACC + gadget decomposition, layout A; digits lifted to [q-512, q+511]
    uint32_t D[4][16];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int j = L + 64 * r;
            const int si = (j - a) & (k2N - 1);
            const uint32_t v = sh.acc[c][si & (kN - 1)];
            const uint32_t rot = (si & kN) ? 0u - v : v;
            const uint32_t t = rot - sh.acc[c][j] + kDecompOffset;
            D[2 * c][r] = ((t >> 22) & 1023u) + (q - 512u);
            D[2 * c + 1][r] = ((t >> 12) & 1023u) + (q - 512u);
        }
    ntt_fwd<4>(D, sc, g.tu_f + 16 * s, g.ts_f + s * 27 * 64 + L, L, q);
    // pointwise MAC with BK_i (layout C: reg r = 4 v + e <-> j = 16 L + r)
#ifdef TFHE_AMD_DIAG_BK
    const uint4 *bk4 = reinterpret_cast<const uint4 *>(g.bk + ((size_t)(0 * 2 + s) * 8) * kN) + L;
#else
    const uint4 *bk4 = reinterpret_cast<const uint4 *>(g.bk + ((size_t)(i * 2 + s) * 8) * kN) + L;
#endif
    const uint32_t qinv = s ? g.qinv_neg1 : g.qinv_neg0;
    uint32_t O[2][16];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            uint4 b[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
#ifdef TFHE_AMD_BK_NT
                typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
                const u32x4_t t = __builtin_nontemporal_load(
                    reinterpret_cast<const u32x4_t *>(&bk4[(c * 4 + p) * 256 + v * 64]));
                b[p] = make_uint4(t.x, t.y, t.z, t.w);
#else
                b[p] = bk4[(c * 4 + p) * 256 + v * 64];
#endif
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t b0 = e == 0 ? b[0].x : e == 1 ? b[0].y : e == 2 ? b[0].z : b[0].w;
                const uint32_t b1 = e == 0 ? b[1].x : e == 1 ? b[1].y : e == 2 ? b[1].z : b[1].w;
                const uint32_t b2 = e == 0 ? b[2].x : e == 1 ? b[2].y : e == 2 ? b[2].z : b[2].w;
                const uint32_t b3 = e == 0 ? b[3].x : e == 1 ? b[3].y : e == 2 ? b[3].z : b[3].w;
                const int r = 4 * v + e;
                const uint64_t x = (uint64_t)D[0][r] * b0 + (uint64_t)D[1][r] * b1 + (uint64_t)D[2][r] * b2 +
                                   (uint64_t)D[3][r] * b3;                          // < 88 q^2 < 2^61
                const uint32_t m = (uint32_t)x * qinv;
                const uint32_t t = (uint32_t)((x + (uint64_t)m * q) >> 32);    // < 3.75 q
                O[c][r] = umin32(t, t - q2);                                     // [0, 2q)
            }
        }
    }
    ntt_inv<2>(O, sc, g.tu_i + 16 * s, g.ts_i + s * 18 * 64 + L, L, q);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) O[c][r] = umin32(O[c][r], O[c][r] - q);   // [0, q)
    if (s == 0) crt_give<0>(sh, O, L);
    else crt_give<1>(sh, O, L);
    __syncthreads();
    if (s == 0) crt_take<0>(sh, O, L, g);
    else crt_take<1>(sh, O, L, g);
    __syncthreads();
}

#ifndef TFHE_AMD_V2_MINW
#define TFHE_AMD_V2_MINW 1     // waves/SIMD floor for the register allocator (A/B builds: 2, 3)
#endif
#ifdef TFHE_AMD_EXPERIMENTAL   // v2 / v3 kernels (EXPERIMENTAL=1 builds)
__global__ __launch_bounds__(kV2Threads, TFHE_AMD_V2_MINW) void k_blind_rotate_v2(V2Args g, int B, BrInput in0, BrInput in1,
                                                                int32_t mu, int32_t *__restrict__ u_a,
                                                                int32_t *__restrict__ u_b) {
    __shared__ V2Shared sh;
    const int tid = threadIdx.x;
    const int s = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = tid & 63;
    const int gct = blockIdx.x;
    const int half = gct >= B;
    const int idx = half ? gct - B : gct;
    const BrInput &in = half ? in1 : in0;

    // gate prologue + modulus switching (boot-gates.cu:98-397; lwe-bootstrapping-functions-fft.cu:1851-1858)
    for (int i = tid; i < kn; i += kV2Threads) {
        uint32_t x = (uint32_t)in.sa * (uint32_t)in.x_a[(size_t)idx * kn + i];
        if (in.sb) x += (uint32_t)in.sb * (uint32_t)in.y_a[(size_t)idx * kn + i];
        sh.bara[i] = modswitch_2N(x);
    }
    if (tid == 0) {
        uint32_t xb = (uint32_t)in.c + (uint32_t)in.sa * (uint32_t)in.x_b[idx];
        if (in.sb) xb += (uint32_t)in.sb * (uint32_t)in.y_b[idx];
        sh.barb = modswitch_2N(xb);
    }
    __syncthreads();
    {   // ACC = (0, X^{2N - barb} (mu, ..., mu))   (:1427-1431)
        const int e = (k2N - sh.barb) & (k2N - 1);
        for (int j = tid; j < kN; j += kV2Threads) {
            sh.acc[0][j] = 0;
            const int si = (j - e) & (k2N - 1);
            sh.acc[1][j] = si < kN ? (uint32_t)mu : 0u - (uint32_t)mu;
        }
    }
    __syncthreads();
    for (int i = 0; i < kn; ++i) {
        const int a = sh.bara[i];
        if (a == 0) continue;            // X^0 - 1 = 0: identity CMux (:705)
        cmux_v2(sh, g, i, a, s, L);
    }
    // sample extraction at index 0 (lwe.cu:41-56)
    int32_t *ua = u_a + (size_t)gct * kN;
    for (int j = tid; j < kN; j += kV2Threads)
        ua[j] = (int32_t)(j == 0 ? sh.acc[0][0] : 0u - sh.acc[0][kN - j]);
    if (tid == 0) u_b[gct] = (int32_t)sh.acc[1][0];
}

__global__ __launch_bounds__(kV2Threads) void k_blind_rotate_v2_debug(V2Args g, int iters, int32_t *__restrict__ acc,
                                                                      const int32_t *__restrict__ bara) {
    __shared__ V2Shared sh;
    const int tid = threadIdx.x;
    const int s = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = tid & 63;
    int32_t *accg = acc + (size_t)blockIdx.x * 2 * kN;
    for (int j = tid; j < 2 * kN; j += kV2Threads) sh.acc[j >> kLogN][j & (kN - 1)] = (uint32_t)accg[j];
    for (int i = tid; i < iters; i += kV2Threads) sh.bara[i] = bara[(size_t)blockIdx.x * iters + i] & (k2N - 1);
    __syncthreads();
    for (int i = 0; i < iters; ++i) {
        const int a = sh.bara[i];
        if (a == 0) continue;
        cmux_v2(sh, g, i, a, s, L);
    }
    for (int j = tid; j < 2 * kN; j += kV2Threads) accg[j] = (int32_t)sh.acc[j >> kLogN][j & (kN - 1)];
}

// ================================================================= v3
// 4 waves per ciphertext: wave w = (s = w & 1: prime, h = w >> 1: accumulator poly).  Wave
// (s, h) decomposes ACC poly h into its 2 digit polys, runs their forward NTTs mod q_s, forms
// the partial MAC of those 2 rows for BOTH output polys, trades the partial for output
// 1 - h with wave (s, 1 - h) through LDS, and runs ONE inverse NTT (output poly h).  Waves
// (0, h) and (1, h) then meet in the CRT exchange.  Half the registers of v2 per wave, so
// twice the waves per SIMD at the same batch, and half the dependent work per CMux step.
constexpr int kV3Threads = 256;

struct V3Shared {
    uint32_t acc[2][kN];
    uint32_t scratch[4][kPadRow];      // one per wave
    int bara[512];
    int barb;
};

template <int S>
__device__ __forceinline__ void crt3_give(V3Shared &sh, int w, const uint32_t (&O)[16], int L) {
    uint32_t *mine = sh.scratch[w];
    constexpr int give = 8 * (1 - S);
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) mine[rr * 64 + L] = O[give + rr];
}
template <int S>
__device__ __forceinline__ void crt3_take(V3Shared &sh, int w, int h, const uint32_t (&O)[16], int L,
                                          const V2Args &g) {
    const uint32_t *other = sh.scratch[w ^ 1];          // wave (1 - s, h)
    constexpr int keep = 8 * S;
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
        const uint32_t xo = other[rr * 64 + L];
        const uint32_t xm = O[keep + rr];
        const uint32_t x0 = S == 0 ? xm : xo, x1 = S == 0 ? xo : xm;
        sh.acc[h][L + 64 * (keep + rr)] += crt_torus(x0, x1, g.crt_h, g.crt_hp);
    }
}

__device__ __forceinline__ void cmux_v3(V3Shared &sh, const V2Args &g, int i, int a, int w, int L) {
    const int s = w & 1, h = w >> 1;
    const uint32_t q = s ? kQ1 : kQ0;
    const uint32_t q2 = 2 * q;
    uint32_t *sc = sh.scratch[w];
    uint32_t D[2][16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int j = L + 64 * r;
        const int si = (j - a) & (k2N - 1);
        const uint32_t v = sh.acc[h][si & (kN - 1)];
        const uint32_t rot = (si & kN) ? 0u - v : v;
        const uint32_t t = rot - sh.acc[h][j] + kDecompOffset;
        D[0][r] = ((t >> 22) & 1023u) + (q - 512u);
        D[1][r] = ((t >> 12) & 1023u) + (q - 512u);
    }
    ntt_fwd<2>(D, sc, g.tu_f + 16 * s, g.ts_f + s * 27 * 64 + L, L, q);
    // partial MAC over rows p = 2h, 2h + 1 for output h (kept) and 1 - h (given away)
    const uint4 *bk4 = reinterpret_cast<const uint4 *>(g.bk + ((size_t)(i * 2 + s) * 8) * kN) + L;
    const uint32_t qinv = s ? g.qinv_neg1 : g.qinv_neg0;
    uint32_t Pk[16], Pg[16];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
            const int c = cc == 0 ? h : 1 - h;
            const uint4 b0 = bk4[(c * 4 + 2 * h) * 256 + v * 64];
            const uint4 b1 = bk4[(c * 4 + 2 * h + 1) * 256 + v * 64];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t x0 = e == 0 ? b0.x : e == 1 ? b0.y : e == 2 ? b0.z : b0.w;
                const uint32_t x1 = e == 0 ? b1.x : e == 1 ? b1.y : e == 2 ? b1.z : b1.w;
                const int r = 4 * v + e;
                const uint64_t x = (uint64_t)D[0][r] * x0 + (uint64_t)D[1][r] * x1;   // < 44 q^2
                const uint32_t m = (uint32_t)x * qinv;
                const uint32_t t = (uint32_t)((x + (uint64_t)m * q) >> 32);        // < 2.4 q
                if (cc == 0) Pk[r] = umin32(t, t - q2);
                else Pg[r] = umin32(t, t - q2);
            }
        }
    }
    // trade partials with wave (s, 1 - h): same lane / register <-> same NTT index j
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[r * 64 + L] = Pg[r];
    __syncthreads();
    const uint32_t *po = sh.scratch[w ^ 2];
    uint32_t O[1][16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t t = Pk[r] + po[r * 64 + L];                 // < 4q
        O[0][r] = umin32(t, t - q2);
    }
    __syncthreads();                                               // partner done with my scratch
    ntt_inv<1>(O, sc, g.tu_i + 16 * s, g.ts_i + s * 18 * 64 + L, L, q);
#pragma unroll
    for (int r = 0; r < 16; ++r) O[0][r] = umin32(O[0][r], O[0][r] - q);   // [0, q)
    if (s == 0) crt3_give<0>(sh, w, O[0], L);
    else crt3_give<1>(sh, w, O[0], L);
    __syncthreads();
    if (s == 0) crt3_take<0>(sh, w, h, O[0], L, g);
    else crt3_take<1>(sh, w, h, O[0], L, g);
    __syncthreads();
}

template <int MINW>
__global__ __launch_bounds__(kV3Threads, MINW) void k_blind_rotate_v3(V2Args g, int B, BrInput in0, BrInput in1,
                                                                int32_t mu, int32_t *__restrict__ u_a,
                                                                int32_t *__restrict__ u_b) {
    __shared__ V3Shared sh;
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = tid & 63;
    const int gct = blockIdx.x;
    const int half = gct >= B;
    const int idx = half ? gct - B : gct;
    const BrInput &in = half ? in1 : in0;
    for (int i = tid; i < kn; i += kV3Threads) {
        uint32_t x = (uint32_t)in.sa * (uint32_t)in.x_a[(size_t)idx * kn + i];
        if (in.sb) x += (uint32_t)in.sb * (uint32_t)in.y_a[(size_t)idx * kn + i];
        sh.bara[i] = modswitch_2N(x);
    }
    if (tid == 0) {
        uint32_t xb = (uint32_t)in.c + (uint32_t)in.sa * (uint32_t)in.x_b[idx];
        if (in.sb) xb += (uint32_t)in.sb * (uint32_t)in.y_b[idx];
        sh.barb = modswitch_2N(xb);
    }
    __syncthreads();
    {
        const int e = (k2N - sh.barb) & (k2N - 1);
        for (int j = tid; j < kN; j += kV3Threads) {
            sh.acc[0][j] = 0;
            const int si = (j - e) & (k2N - 1);
            sh.acc[1][j] = si < kN ? (uint32_t)mu : 0u - (uint32_t)mu;
        }
    }
    __syncthreads();
    for (int i = 0; i < kn; ++i) {
        const int a = sh.bara[i];
        if (a == 0) continue;
        cmux_v3(sh, g, i, a, w, L);
    }
    int32_t *ua = u_a + (size_t)gct * kN;
    for (int j = tid; j < kN; j += kV3Threads)
        ua[j] = (int32_t)(j == 0 ? sh.acc[0][0] : 0u - sh.acc[0][kN - j]);
    if (tid == 0) u_b[gct] = (int32_t)sh.acc[1][0];
}

__global__ __launch_bounds__(kV3Threads, 3) void k_blind_rotate_v3_debug(V2Args g, int iters, int32_t *__restrict__ acc,
                                                                      const int32_t *__restrict__ bara) {
    __shared__ V3Shared sh;
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = tid & 63;
    int32_t *accg = acc + (size_t)blockIdx.x * 2 * kN;
    for (int j = tid; j < 2 * kN; j += kV3Threads) sh.acc[j >> kLogN][j & (kN - 1)] = (uint32_t)accg[j];
    for (int i = tid; i < iters; i += kV3Threads) sh.bara[i] = bara[(size_t)blockIdx.x * iters + i] & (k2N - 1);
    __syncthreads();
    for (int i = 0; i < iters; ++i) {
        const int a = sh.bara[i];
        if (a == 0) continue;
        cmux_v3(sh, g, i, a, w, L);
    }
    for (int j = tid; j < 2 * kN; j += kV3Threads) accg[j] = (int32_t)sh.acc[j >> kLogN][j & (kN - 1)];
}

// BK (coefficient domain [i][p][c][N]) -> v2 layout [i][s][c][p][v][L][e], j = 16 L + 4 v + e,
// from the v1 NTT-domain key [i][s][p][c][N] (same values, bit-reversed NTT order j)
#endif  // TFHE_AMD_EXPERIMENTAL

__global__ __launch_bounds__(256) void k_bk_v1_to_v2(const uint32_t *__restrict__ v1, uint32_t *__restrict__ v2) {
    const int poly = blockIdx.x;   // (i*2 + s)*8 + c*4 + p
    const int p = poly & 3, c = (poly >> 2) & 1, is = poly >> 3;
    const uint32_t *src = v1 + ((size_t)is * 8 + p * 2 + c) * kN;
    uint32_t *dst = v2 + (size_t)poly * kN;
    for (int j = threadIdx.x; j < kN; j += blockDim.x) {
        const int L = j >> 4, v = (j >> 2) & 3, e = j & 3;
        dst[v * 256 + L * 4 + e] = src[j];
    }
}

}  // namespace

// Twiddle tables of the v2 kernel, generated on the host in the kernel's consumption order.
void build_v2_twiddles(const NttTables &t, uint2 *tu_f, uint2 *tu_i, uint2 *ts_f, uint2 *ts_i) {
    for (int s = 0; s < 2; ++s) {
        for (int idx = 0; idx < 16; ++idx) {
            tu_f[s * 16 + idx] = make_uint2(0u - t.psi[s][idx], t.psip[s][idx]);   // negated: bf_ct
            tu_i[s * 16 + idx] = make_uint2(t.ipsi[s][idx], t.ipsip[s][idx]);
        }
        int slot = 0;
        for (int K = 5; K >= 2; --K)
            for (int g = 0; g < (1 << (5 - K)); ++g, ++slot)
                for (int L = 0; L < 64; ++L) {
                    const int idx = (1 << (9 - K)) + ((L >> 2) << (5 - K)) + g;
                    ts_f[(s * 27 + slot) * 64 + L] = make_uint2(0u - t.psi[s][idx], t.psip[s][idx]);
                }
        for (int K = 1; K >= 0; --K)
            for (int g = 0; g < (1 << (3 - K)); ++g, ++slot)
                for (int L = 0; L < 64; ++L) {
                    const int idx = (1 << (9 - K)) + (L << (3 - K)) + g;
                    ts_f[(s * 27 + slot) * 64 + L] = make_uint2(0u - t.psi[s][idx], t.psip[s][idx]);
                }
        slot = 0;
        for (int K = 0; K <= 3; ++K)
            for (int g = 0; g < (1 << (3 - K)); ++g, ++slot)
                for (int L = 0; L < 64; ++L) {
                    const int idx = (1 << (9 - K)) + (L << (3 - K)) + g;
                    ts_i[(s * 18 + slot) * 64 + L] = make_uint2(t.ipsi[s][idx], t.ipsip[s][idx]);
                }
        for (int K = 4; K <= 5; ++K)
            for (int g = 0; g < (1 << (5 - K)); ++g, ++slot)
                for (int L = 0; L < 64; ++L) {
                    const int idx = (1 << (9 - K)) + ((L >> 2) << (5 - K)) + g;
                    ts_i[(s * 18 + slot) * 64 + L] = make_uint2(t.ipsi[s][idx], t.ipsip[s][idx]);
                }
    }
}

static V2Args v2_args(const DeviceKey &key) {
    V2Args g;
    g.bk = key.bk_v2;
    g.tu_f = key.tw2;
    g.tu_i = key.tw2 + 32;
    g.ts_f = key.tw2 + 64;
    g.ts_i = key.tw2 + 64 + 2 * 27 * 64;
    g.qinv_neg0 = key.qinv_neg[0];
    g.qinv_neg1 = key.qinv_neg[1];
    g.crt_h = key.crt_h;
    g.crt_hp = key.crt_hp;
    return g;
}

hipError_t launch_bk_v1_to_v2(const uint32_t *d_v1, uint32_t *d_v2, hipStream_t s) {
    hipLaunchKernelGGL(k_bk_v1_to_v2, dim3(kn * 2 * 8), dim3(256), 0, s, d_v1, d_v2);
    return hipGetLastError();
}

#ifdef TFHE_AMD_EXPERIMENTAL   // v2 / v3 launchers
hipError_t launch_blind_rotate_v2(const DeviceKey &key, int B, int halves, const BrInput *in, int32_t mu,
                                  int32_t *u_a, int32_t *u_b, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    const BrInput in1 = halves > 1 ? in[1] : in[0];
    hipLaunchKernelGGL(k_blind_rotate_v2, dim3(B * halves), dim3(kV2Threads), 0, s, v2_args(key), B, in[0], in1, mu,
                       u_a, u_b);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_v3(const DeviceKey &key, int B, int halves, const BrInput *in, int32_t mu,
                                  int32_t *u_a, int32_t *u_b, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    const BrInput in1 = halves > 1 ? in[1] : in[0];
    static const int minw = [] {
        const char *e = getenv("TFHE_AMD_V3W");
        return (e && atoi(e) == 4) ? 4 : 3;
    }();
    if (minw == 4)
        hipLaunchKernelGGL(k_blind_rotate_v3<4>, dim3(B * halves), dim3(kV3Threads), 0, s, v2_args(key), B, in[0], in1,
                           mu, u_a, u_b);
    else
        hipLaunchKernelGGL(k_blind_rotate_v3<3>, dim3(B * halves), dim3(kV3Threads), 0, s, v2_args(key), B, in[0], in1,
                           mu, u_a, u_b);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_v3_debug(const DeviceKey &key, int B, int iters, int32_t *acc, const int32_t *bara,
                                        hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (iters < 0 || iters > kn) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_blind_rotate_v3_debug, dim3(B), dim3(kV3Threads), 0, s, v2_args(key), iters, acc, bara);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_v2_debug(const DeviceKey &key, int B, int iters, int32_t *acc, const int32_t *bara,
                                        hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (iters < 0 || iters > kn) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_blind_rotate_v2_debug, dim3(B), dim3(kV2Threads), 0, s, v2_args(key), iters, acc, bara);
    return hipGetLastError();
}

#endif  // TFHE_AMD_EXPERIMENTAL

}  // namespace tfhe_amd
