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


}  // namespace tfhe_amd
