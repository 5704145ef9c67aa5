// blind_rotate_v7.hip — v6's fp64 FFT external product with the bootstrapping key staged in LDS
// and shared by the ciphertexts of a workgroup.
//
// v6 gives each ciphertext its own 2-wave workgroup, and each wave reads its 32 KB share of
// BK_i per CMux step from L2 into registers (plus 24 KB of twiddles): at B = 1024 that is
// ~450 KB per CU per step through the vector-memory path, and a build that skips the key loads
// runs 12 % faster.  v7 puts C ciphertexts (2C waves) in one workgroup that
// advances in lock-step:
//  * BK_i (64 KB) is copied once per workgroup into LDS by LDS-DMA (`global_load_lds_dwordx4`,
//    no VGPRs), issued right after the step's MAC barrier for step i + 1, so it has the inverse
//    transform, the accumulator update and the next forward transform to land; the C
//    ciphertexts read it from LDS (key traffic through L2 / 4 at C = 4);
//  * the per-lane twiddles live in LDS too (compact 17 KB table), so the loop issues no
//    register-destination global load at all;
//  * three workgroup barriers per step: B1 (the DMA of BK_i has landed), B2 (MAC partial sums
//    stored, every wave done reading BK_i -> the next DMA may start), B3 (the partner wave has
//    read this wave's partial sum, the buffer is free for the inverse transposes);
//  * rotation, decomposition, FFTs, MAC and rounding are v6's (fft_wave.h), so results are
//    bit-identical to v6 (and to the exact NTT generations); a step with bara_i = 0 is executed
//    (its digits are 0, the product is exactly 0) because every wave must reach the barriers.
// LDS at C = 4: 64 KB key + 8 x 9 KB wave buffers + 17 KB twiddles + 4 KB rotation amounts.
#include <cmath>
#include "engine.h"
#include "modarith.h"
#include "fft_wave.h"

namespace tfhe_amd {

namespace {

constexpr int kKeyWords = 4 * 2 * 8 * 64;   // BK_i slice, double2: [row][c][r][L]

template <int C>
struct __attribute__((aligned(16))) V7Shared {
    double2 K[kKeyWords];
    double2 X[2 * C][kXSlots];
    double2 tw[kT7Words];
    short bara[C][512];
    int barb[C];
};
static_assert(sizeof(V7Shared<4>) <= 160 * 1024, "v7 LDS fits a CU");

__device__ __forceinline__ uint32_t lds_addr(const void *p) { return (uint32_t)(uintptr_t)p; }

// one 1 KB LDS-DMA: lane L's 16 B from src (per lane) to LDS dst + 16 L (dst wave-uniform).
// Inline asm so that hipcc neither counts it nor inserts vmcnt(0) in front of unrelated LDS
// reads; completion is waited for explicitly (B1).
__device__ __forceinline__ void glds16(const double2 *src, uint32_t dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(dst)
                 : "memory");
}

// BK_i -> sh.K: 64 chunks of 1 KB, wave wv of the 2C takes chunks wv, wv + 2C, ...
template <int C>
__device__ __forceinline__ void dma_key(V7Shared<C> &sh, const double2 *bk, int i, int wv, int L) {
    const double2 *src = bk + (size_t)i * kKeyWords + L;
    const uint32_t base = lds_addr(sh.K);
#pragma unroll
    for (int m = 0; m < 64 / (2 * C); ++m) {
        const int k = wv + 2 * C * m;
        glds16(src + k * 64, __builtin_amdgcn_readfirstlane(base + k * 1024));
    }
}

__device__ __forceinline__ void barrier_dma() { asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void barrier_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// key rows 2w, 2w + 1 of output c from the LDS slice ([row][c][r][L])
__device__ __forceinline__ void load_bk7(Cx (&b)[2][8], const double2 *K, int w, int c, int L) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        b[0][r] = ld(K + ((2 * w) * 2 + c) * 512 + r * 64 + L);
        b[1][r] = ld(K + ((2 * w + 1) * 2 + c) * 512 + r * 64 + L);
    }
}

// one lock-step CMux step of wave (ciphertext c, polynomial w): acc_w += [(X^a - 1) ACC] (x) BK_i
template <int C>
__device__ __forceinline__ void cmux_v7(V7Shared<C> &sh, const double2 *bk, const Tw4 &tA, int i, int iters,
                                        int a, int wv, int w, int L, uint32_t (&acc)[16]) {
    double2 *X = sh.X[wv];
    uint32_t *E = reinterpret_cast<uint32_t *>(X);
    write_ext(E, acc, L);
    wave_sync();
    Cx D[2][8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int base = (L + 256 * q - a) & (k2N - 1);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int r = 4 * q + rr;
            const uint32_t diff = E[base + 64 * rr] - acc[r];
            const int32_t hi = (int32_t)(diff + (kDecompOffset + 0x80000000u)) >> 22;
            const int32_t lo = __builtin_amdgcn_sbfe((int32_t)(diff + (kDecompOffset + 0x200000u)), 12, 10);
            if (r < 8) {
                D[0][r].re = (double)hi;
                D[1][r].re = (double)lo;
            } else {
                D[0][r - 8].im = (double)hi;
                D[1][r - 8].im = (double)lo;
            }
        }
    }
    wave_sync();
    fft_fwd_AB_t<2>(D, X, tA, tw7_fwdB(sh.tw, L), L);
    const Tw4 tC = tw7_fwdC(sh.tw, L);
    barrier_dma();                                   // B1: BK_i is in sh.K
    Cx Y[8];
    Cx bv[2][8];
    load_bk7(bv, sh.K, w, 1 - w, L);
    fft_fwd_C<2>(D, tC);
    mac6(D, bv, Y);
    load_bk7(bv, sh.K, w, w, L);
    store_C(X, Y, L);                                // partial sum of output 1 - w for the partner
    mac6(D, bv, Y);
    barrier_lds();                                   // B2: partials stored, BK_i fully read
    if (i + 1 < iters) dma_key(sh, bk, i + 1, wv, L);
    // inverse: LDS read groups issued whole before their arithmetic (as in v6)
    {
        Cx o[8];
        load_C(sh.X[wv ^ 1], o, L);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            Y[r].re += o[r].re;
            Y[r].im += o[r].im;
        }
    }
    pass_dit_C(Y);
    const Tw4 tB = tw7_invB(sh.tw, L);
    barrier_lds();                                   // B3: the partner has read X[wv]
    store_C(X, Y, L);
    wave_sync();
    load_B_p(X, Y, L);
    __builtin_amdgcn_sched_barrier(0);
    pass_dit(Y, tB.w0, tB.w1, tB.w2a, tB.w2b);
    {
        const Tw4 tI = tw7_invA(sh.tw, L);
        Cx z[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) z[r] = ld(sh.tw + kT7Post + r * 64 + L);
        wave_sync();
        store_B_ab(X, Y, L);
        wave_sync();
        load_A(X, Y, L);
        __builtin_amdgcn_sched_barrier(0);
        pass_dit(Y, tI.w0, tI.w1, tI.w2a, tI.w2b);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const double re = fma_(Y[r].re, z[r].re, -(Y[r].im * z[r].im));
            const double im = fma_(Y[r].re, z[r].im, Y[r].im * z[r].re);
            Y[r] = Cx{re, im};
        }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        acc[r] += torus_of(Y[r].re);
        acc[r + 8] += torus_of(Y[r].im);
    }
    wave_sync();
}

// workgroup prologue shared by all v7 kernels: twiddles to LDS, DMA of BK_0
template <int C>
__device__ __forceinline__ void v7_prologue(V7Shared<C> &sh, const double2 *bk, const double2 *tw, int iters,
                                            int wv, int L) {
    for (int e = threadIdx.x; e < kT7Words; e += 128 * C) sh.tw[e] = tw[t7_src(e)];
    if (iters > 0) dma_key(sh, bk, 0, wv, L);
}

template <int C>
__device__ __forceinline__ void v7_loop(V7Shared<C> &sh, const double2 *bk, const Tw4 &tA, int iters, int c, int wv,
                                        int w, int L, uint32_t (&acc)[16]) {
    int a = sh.bara[c][0];
    for (int i = 0; i < iters; ++i) {
        const int a_next = sh.bara[c][i + 1 < iters ? i + 1 : i];   // read a step ahead
        cmux_v7<C>(sh, bk, tA, i, iters, a, wv, w, L, acc);
        a = a_next;
    }
}

// gate prologue + modulus switching of ciphertext slot c (its 128 threads), :1851-1858
template <int C>
__device__ __forceinline__ void v7_modswitch(V7Shared<C> &sh, const RowTerms6 &t, bool valid, int c, int tc) {
    for (int i = tc; i < kn; i += 128) {
        uint32_t x = 0;
        if (valid) {   // a circuit row may have no x wire (constant rows): null like y / z
            if (t.xa) x = (uint32_t)t.sa * (uint32_t)t.xa[i];
            if (t.ya) x += (uint32_t)t.sb * (uint32_t)t.ya[i];
            if (t.za) x += (uint32_t)t.sc * (uint32_t)t.za[i];
        }
        sh.bara[c][i] = (short)modswitch_2N(x);
    }
    if (tc == 0) {
        uint32_t xb = 0;
        if (valid) {
            xb = (uint32_t)t.c;
            if (t.xb) xb += (uint32_t)t.sa * (uint32_t)t.xb[0];
            if (t.yb) xb += (uint32_t)t.sb * (uint32_t)t.yb[0];
            if (t.zb) xb += (uint32_t)t.sc * (uint32_t)t.zb[0];
        }
        sh.barb[c] = modswitch_2N(xb);
    }
}

template <int C>
__global__ __launch_bounds__(128 * C, C == 4 ? 2 : 1) void k_blind_rotate_v7(const double2 *__restrict__ bk,
                                                                const double2 *__restrict__ tw, int B, int nct,
                                                                BrInput in0, BrInput in1, int32_t mu,
                                                                int32_t *__restrict__ u_a, int32_t *__restrict__ u_b) {
    __shared__ V7Shared<C> sh;
    const int tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = wv >> 1, w = wv & 1, L = tid & 63;
    const int gct = blockIdx.x * C + c;          // ciphertext index in [0, halves * B)
    const bool valid = gct < nct;
    v7_prologue<C>(sh, bk, tw, kn, wv, L);
    {
        const int half = gct >= B;
        const int idx = half ? gct - B : gct;
        const BrInput &in = half ? in1 : in0;
        RowTerms6 t;
        t.c = in.c; t.sa = in.sa; t.sb = in.sb; t.sc = 0;
        t.xa = in.x_a + (size_t)idx * kn; t.xb = in.x_b + idx;
        t.ya = in.sb ? in.y_a + (size_t)idx * kn : nullptr; t.yb = in.sb ? in.y_b + idx : nullptr;
        t.za = nullptr; t.zb = nullptr;
        v7_modswitch<C>(sh, t, valid, c, tid & 127);
    }
    const Tw4 tA = load_tw_sgpr(tw);
    __syncthreads();
    uint32_t acc[16];
    {
        const int e = (k2N - sh.barb[c]) & (k2N - 1);
#pragma unroll
        for (int r = 0; r < 16; ++r)
            acc[r] = w == 0 ? 0u : (((L + 64 * r - e) & (k2N - 1)) < kN ? (uint32_t)mu : 0u - (uint32_t)mu);
    }
    v7_loop<C>(sh, bk, tA, kn, c, wv, w, L, acc);
    if (!valid) return;
    if (w == 0) {
        uint32_t *E = reinterpret_cast<uint32_t *>(sh.X[wv]);
        write_ext(E, acc, L);
        wave_sync();
        int32_t *ua = u_a + (size_t)gct * kN;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int j = L + 64 * r;
            ua[j] = (int32_t)E[(k2N - j) & (k2N - 1)];
        }
    } else if (L == 0) {
        u_b[gct] = (int32_t)acc[0];
    }
}

template <int C>
__global__ __launch_bounds__(128 * C, C == 4 ? 2 : 1) void k_blind_rotate_v7_rows(const double2 *__restrict__ bk,
                                                                     const double2 *__restrict__ tw, int B,
                                                                     const CircRow *__restrict__ rows,
                                                                     const int32_t *__restrict__ wa,
                                                                     const int32_t *__restrict__ wb, int32_t mu,
                                                                     int32_t *__restrict__ u_a,
                                                                     int32_t *__restrict__ u_b) {
    __shared__ V7Shared<C> sh;
    const int tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = wv >> 1, w = wv & 1, L = tid & 63;
    const int k = blockIdx.x * C + c, r = blockIdx.y;
    const bool valid = k < B;
    v7_prologue<C>(sh, bk, tw, kn, wv, L);
    {
        const CircRow row = rows[r];
        auto wire = [&](int wi, const int32_t *&pa, const int32_t *&pb) {
            if (wi < 0) { pa = nullptr; pb = nullptr; return; }
            const size_t slot = (size_t)wi * B + k;
            pa = wa + slot * kn;
            pb = wb + slot;
        };
        RowTerms6 t;
        t.c = row.c; t.sa = row.sa; t.sb = row.sb; t.sc = row.sc;
        wire(row.x, t.xa, t.xb);
        wire(row.y, t.ya, t.yb);
        wire(row.z, t.za, t.zb);
        v7_modswitch<C>(sh, t, valid, c, tid & 127);
    }
    const Tw4 tA = load_tw_sgpr(tw);
    __syncthreads();
    uint32_t acc[16];
    {
        const int e = (k2N - sh.barb[c]) & (k2N - 1);
#pragma unroll
        for (int rr = 0; rr < 16; ++rr)
            acc[rr] = w == 0 ? 0u : (((L + 64 * rr - e) & (k2N - 1)) < kN ? (uint32_t)mu : 0u - (uint32_t)mu);
    }
    v7_loop<C>(sh, bk, tA, kn, c, wv, w, L, acc);
    if (!valid) return;
    const size_t slot = (size_t)r * B + k;
    if (w == 0) {
        uint32_t *E = reinterpret_cast<uint32_t *>(sh.X[wv]);
        write_ext(E, acc, L);
        wave_sync();
        int32_t *ua = u_a + slot * kN;
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
            const int j = L + 64 * rr;
            ua[j] = (int32_t)E[(k2N - j) & (k2N - 1)];
        }
    } else if (L == 0) {
        u_b[slot] = (int32_t)acc[0];
    }
}

// explicit CMux steps on accumulators acc [B][2][kN] with rotation amounts bara [B][iters]
template <int C>
__global__ __launch_bounds__(128 * C, C == 4 ? 2 : 1) void k_blind_rotate_v7_debug(const double2 *__restrict__ bk,
                                                                      const double2 *__restrict__ tw, int B, int iters,
                                                                      int32_t *__restrict__ acc,
                                                                      const int32_t *__restrict__ bara) {
    __shared__ V7Shared<C> sh;
    const int tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = wv >> 1, w = wv & 1, L = tid & 63;
    const int g = blockIdx.x * C + c;
    const bool valid = g < B;
    v7_prologue<C>(sh, bk, tw, iters, wv, L);
    for (int i = tid & 127; i < iters; i += 128)
        sh.bara[c][i] = valid ? (short)(bara[(size_t)g * iters + i] & (k2N - 1)) : (short)0;
    uint32_t ac[16];
    int32_t *accg = acc + (size_t)(valid ? g : 0) * 2 * kN + (size_t)w * kN;
#pragma unroll
    for (int r = 0; r < 16; ++r) ac[r] = valid ? (uint32_t)accg[L + 64 * r] : 0u;
    const Tw4 tA = load_tw_sgpr(tw);
    __syncthreads();
    v7_loop<C>(sh, bk, tA, iters, c, wv, w, L, ac);
    if (!valid) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) accg[L + 64 * r] = (int32_t)ac[r];
}

// ciphertexts per workgroup: 4 once every CU gets one workgroup, fewer for small launches
int v7_group(int nct) { return nct >= 768 ? 4 : nct > 256 ? 2 : 1; }

}  // namespace

hipError_t launch_blind_rotate_v7(const DeviceKey &key, int B, int halves, const BrInput *in, int32_t mu,
                                  int32_t *u_a, int32_t *u_b, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (!key.bk_fft) return hipErrorInvalidValue;
    const BrInput in1 = halves > 1 ? in[1] : in[0];
    const int nct = B * halves, C = v7_group(nct);
    const dim3 grid((nct + C - 1) / C);
    if (C == 4)
        hipLaunchKernelGGL(k_blind_rotate_v7<4>, grid, dim3(512), 0, s, key.bk_fft, key.tw6, B, nct, in[0], in1, mu,
                           u_a, u_b);
    else if (C == 2)
        hipLaunchKernelGGL(k_blind_rotate_v7<2>, grid, dim3(256), 0, s, key.bk_fft, key.tw6, B, nct, in[0], in1, mu,
                           u_a, u_b);
    else
        hipLaunchKernelGGL(k_blind_rotate_v7<1>, grid, dim3(128), 0, s, key.bk_fft, key.tw6, B, nct, in[0], in1, mu,
                           u_a, u_b);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_v7_rows(const DeviceKey &key, int B, int nrows, const CircRow *rows, const int32_t *wa,
                                       const int32_t *wb, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t s) {
    if (B <= 0 || nrows <= 0) return hipSuccess;
    if (nrows > 65535 || !key.bk_fft) return hipErrorInvalidValue;
    int C = v7_group(B * nrows);      // no more slots per workgroup than instances
    while (C > B) C >>= 1;
    const dim3 grid((B + C - 1) / C, nrows);
    if (C == 4)
        hipLaunchKernelGGL(k_blind_rotate_v7_rows<4>, grid, dim3(512), 0, s, key.bk_fft, key.tw6, B, rows, wa, wb, mu,
                           u_a, u_b);
    else if (C == 2)
        hipLaunchKernelGGL(k_blind_rotate_v7_rows<2>, grid, dim3(256), 0, s, key.bk_fft, key.tw6, B, rows, wa, wb, mu,
                           u_a, u_b);
    else
        hipLaunchKernelGGL(k_blind_rotate_v7_rows<1>, grid, dim3(128), 0, s, key.bk_fft, key.tw6, B, rows, wa, wb, mu,
                           u_a, u_b);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_v7_debug(const DeviceKey &key, int B, int iters, int32_t *acc, const int32_t *bara,
                                        hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (iters < 0 || iters > kn || !key.bk_fft) return hipErrorInvalidValue;
    // C = 2 even for tiny batches so that the lock-step / shared-key path is what the test sees
    hipLaunchKernelGGL(k_blind_rotate_v7_debug<2>, dim3((B + 1) / 2), dim3(256), 0, s, key.bk_fft, key.tw6, B, iters,
                       acc, bara);
    return hipGetLastError();
}

}  // namespace tfhe_amd
