// fft_wave.h — one wave's share of the fp64 negacyclic FFT external product (v6 blind
// rotation): complex type, butterflies, the three radix-8 register passes and their LDS
// transposes, twiddle tables, the mod-2^32 rounding and the key MAC.  Design: DESIGN.md §3,
// emulation: scripts/emu_v6.py.
#pragma once
#include "engine.h"

namespace tfhe_amd {
namespace {

constexpr int kExt6 = 2240;          // 2N + 192: quarter bases (< 2N) + 64 * 3
constexpr int kXSlots = 576;         // 512 complex + pad (slot map of the B <-> C transposes)

struct Cx {
    double re, im;
};

// twiddle table (double2): [0, 4) forward pass A (uniform), [4, 260) forward pass B [4][64],
// [260, 516) forward pass C, [516, 772) inverse pass B [4][64], [772, 1028) inverse pass A,
// [1028, 1540) post-twist zeta^-(L + 64 r) [8][64]
constexpr int kTwInv = 516;
constexpr int kTwPost = 1028;
// [1540, 1604) zeta^-L, [1604, 1668) the inverse pass-A twiddle a times zeta^-L (cmux_v6's folded
// post-twist)
constexpr int kTwSig = 1540;
constexpr int kTwInvAs = 1604;

__device__ __forceinline__ double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }

// (u, v) -> (u + W v, u - W v), W = w (ODD = false) or i w (ODD = true); 6 fp64 ops
template <bool ODD>
__device__ __forceinline__ void bf_fwd(Cx &u, Cx &v, const Cx &w) {
    double xr, xi;
    if (!ODD) {
        xr = fma_(w.re, v.re, u.re);
        xr = fma_(-w.im, v.im, xr);
        xi = fma_(w.re, v.im, u.im);
        xi = fma_(w.im, v.re, xi);
    } else {
        xr = fma_(-w.re, v.im, u.re);
        xr = fma_(-w.im, v.re, xr);
        xi = fma_(w.re, v.re, u.im);
        xi = fma_(-w.im, v.im, xi);
    }
    v.re = fma_(2.0, u.re, -xr);
    v.im = fma_(2.0, u.im, -xi);
    u.re = xr;
    u.im = xi;
}

// one radix-8 register pass: CT stages at register distance 4, 2, 1
template <int NP>
__device__ __forceinline__ void pass_fwd(Cx (&x)[NP][8], const Cx &w0, const Cx &w1, const Cx &w2a, const Cx &w2b) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bf_fwd<false>(x[p][r], x[p][r + 4], w0);
        bf_fwd<false>(x[p][0], x[p][2], w1);
        bf_fwd<false>(x[p][1], x[p][3], w1);
        bf_fwd<true>(x[p][4], x[p][6], w1);
        bf_fwd<true>(x[p][5], x[p][7], w1);
        bf_fwd<false>(x[p][0], x[p][1], w2a);
        bf_fwd<true>(x[p][2], x[p][3], w2a);
        bf_fwd<false>(x[p][4], x[p][5], w2b);
        bf_fwd<true>(x[p][6], x[p][7], w2b);
    }
}

// inverse: radix-2 DIT on the forward's bit-reversed output (slot n holds the evaluation at
// zeta omega^brv9(n)), natural order out, then the zeta^-n post-twist (scripts/emu_v6.py
// check_dit).  One register pass: stages at register distance 1, 2, 4 with per-lane twiddles
// a, b (and -i b), c, c2 (and -i c, -i c2).
__device__ __forceinline__ Cx negi_(const Cx &w) { return Cx{-w.re, -w.im}; }   // i (-w) = -i w
__device__ __forceinline__ void pass_dit(Cx (&x)[8], const Cx &a, const Cx &b, const Cx &c, const Cx &c2) {
    bf_fwd<false>(x[0], x[1], a);
    bf_fwd<false>(x[2], x[3], a);
    bf_fwd<false>(x[4], x[5], a);
    bf_fwd<false>(x[6], x[7], a);
    bf_fwd<false>(x[0], x[2], b);
    bf_fwd<true>(x[1], x[3], negi_(b));
    bf_fwd<false>(x[4], x[6], b);
    bf_fwd<true>(x[5], x[7], negi_(b));
    bf_fwd<false>(x[0], x[4], c);
    bf_fwd<false>(x[1], x[5], c2);
    bf_fwd<true>(x[2], x[6], negi_(c));
    bf_fwd<true>(x[3], x[7], negi_(c2));
}
// W = 1 and W = -i butterflies: 4 adds
__device__ __forceinline__ void bf_one(Cx &u, Cx &v) {
    const Cx t = u;
    u.re = t.re + v.re;
    u.im = t.im + v.im;
    v.re = t.re - v.re;
    v.im = t.im - v.im;
}
__device__ __forceinline__ void bf_negi(Cx &u, Cx &v) {   // (u - i v, u + i v)
    const Cx t = u;
    u.re = t.re + v.im;
    u.im = t.im - v.re;
    const double vr = v.re;
    v.re = t.re - v.im;
    v.im = t.im + vr;
}
// pass C of the inverse: stages 0..2 (h = 1, 2, 4), twiddles 1, -i, e^{-i pi / 4}, -i e^{-i pi / 4}
__device__ __forceinline__ void pass_dit_C(Cx (&x)[8]) {
    constexpr double h = 0.70710678118654752440;
    bf_one(x[0], x[1]);
    bf_one(x[2], x[3]);
    bf_one(x[4], x[5]);
    bf_one(x[6], x[7]);
    bf_one(x[0], x[2]);
    bf_negi(x[1], x[3]);
    bf_one(x[4], x[6]);
    bf_negi(x[5], x[7]);
    bf_one(x[0], x[4]);
    bf_fwd<false>(x[1], x[5], Cx{h, -h});
    bf_negi(x[2], x[6]);
    bf_fwd<true>(x[3], x[7], Cx{-h, h});
}

__device__ __forceinline__ Cx cmul(const Cx &a, const Cx &b) {
    return Cx{fma_(a.re, b.re, -(a.im * b.im)), fma_(a.re, b.im, a.im * b.re)};
}
__device__ __forceinline__ Cx ld(const double2 *p) {
    const double2 v = *p;
    return Cx{v.x, v.y};
}
__device__ __forceinline__ void st(double2 *p, const Cx &v) { *p = make_double2(v.re, v.im); }

// per-lane twiddles of pass B (k = 0) or C (k = 1)
struct Tw4 {
    Cx w0, w1, w2a, w2b;
};
__device__ __forceinline__ Tw4 load_tw(const double2 *tw, int k, int L) {
    const double2 *t = tw + 4 + k * 256 + L;
    return Tw4{ld(t), ld(t + 64), ld(t + 128), ld(t + 192)};
}
// inverse DIT twiddles of pass B (k = 0) or A (k = 1): a, b, c, c2
__device__ __forceinline__ Tw4 load_tw_inv(const double2 *tw, int k, int L) {
    const double2 *t = tw + kTwInv + k * 256 + L;
    return Tw4{ld(t), ld(t + 64), ld(t + 128), ld(t + 192)};
}
__device__ __forceinline__ Tw4 load_tw_uniform(const double2 *tw) {
    return Tw4{ld(tw), ld(tw + 1), ld(tw + 2), ld(tw + 3)};
}

// Single-wave LDS exchanges: LDS executes one wave's DS instructions in order; the fences
// keep the compiler from moving a lane's read above another lane's write.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void lds_barrier6() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Slot maps (bank-conflict free for the 16-B accesses):
//   A <-> B transposes: s(n) = n ^ (8 * bit6(n));  B <-> C: s(n) = n + (n >> 3)
// layout A: n = L + 64 r;  B: n = (L & 7) + 8 r + 64 (L >> 3);  C: n = 8 L + r
__device__ __forceinline__ void store_A(double2 *X, const Cx (&x)[8], int L) {
#pragma unroll
    for (int r = 0; r < 8; ++r) st(X + ((L ^ (8 * (r & 1))) + 64 * r), x[r]);
}
__device__ __forceinline__ void load_A(const double2 *X, Cx (&x)[8], int L) {
#pragma unroll
    for (int r = 0; r < 8; ++r) x[r] = ld(X + ((L ^ (8 * (r & 1))) + 64 * r));
}
__device__ __forceinline__ int baseB_ab(int L, int odd) {   // slot of (L, r) = base(r & 1) + 8 r
    const int b = (L >> 3) & 1;
    const int n0 = (L & 7) + 64 * (L >> 3);
    return odd ? n0 - 8 * b : n0 + 8 * b;
}
__device__ __forceinline__ void load_B_ab(const double2 *X, Cx (&x)[8], int L) {
    const int e = baseB_ab(L, 0), o = baseB_ab(L, 1);
#pragma unroll
    for (int r = 0; r < 8; ++r) x[r] = ld(X + ((r & 1) ? o : e) + 8 * r);
}
__device__ __forceinline__ void store_B_ab(double2 *X, const Cx (&x)[8], int L) {
    const int e = baseB_ab(L, 0), o = baseB_ab(L, 1);
#pragma unroll
    for (int r = 0; r < 8; ++r) st(X + ((r & 1) ? o : e) + 8 * r, x[r]);
}
__device__ __forceinline__ void store_B_p(double2 *X, const Cx (&x)[8], int L) {
    const int base = (L & 7) + 72 * (L >> 3);
#pragma unroll
    for (int r = 0; r < 8; ++r) st(X + base + 9 * r, x[r]);
}
__device__ __forceinline__ void load_B_p(const double2 *X, Cx (&x)[8], int L) {
    const int base = (L & 7) + 72 * (L >> 3);
#pragma unroll
    for (int r = 0; r < 8; ++r) x[r] = ld(X + base + 9 * r);
}
__device__ __forceinline__ void store_C(double2 *X, const Cx (&x)[8], int L) {
#pragma unroll
    for (int r = 0; r < 8; ++r) st(X + 9 * L + r, x[r]);
}
__device__ __forceinline__ void load_C(const double2 *X, Cx (&x)[8], int L) {
#pragma unroll
    for (int r = 0; r < 8; ++r) x[r] = ld(X + 9 * L + r);
}

// wave-uniform double -> SGPR pair
__device__ __forceinline__ double uni(double v) {
    const long long bits = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)bits);
    const int hi = __builtin_amdgcn_readfirstlane((int)(bits >> 32));
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ Tw4 load_tw_sgpr(const double2 *tw) {
    Tw4 t = load_tw_uniform(tw);
    t.w0 = Cx{uni(t.w0.re), uni(t.w0.im)};
    t.w1 = Cx{uni(t.w1.re), uni(t.w1.im)};
    t.w2a = Cx{uni(t.w2a.re), uni(t.w2a.im)};
    t.w2b = Cx{uni(t.w2b.re), uni(t.w2b.im)};
    return t;
}

// forward transform of NP polynomials, layout A in -> layout C (slot 8 L + r): passes A and
// B and both transposes; the caller runs pass C (fft_fwd_C) so that it can put loads in
// flight first.  tA = the pass-A (uniform) twiddles, held in SGPRs for the whole kernel.
template <int NP>
__device__ __forceinline__ void fft_fwd_AB(Cx (&x)[NP][8], double2 *X, const double2 *tw, const Tw4 &tA, int L) {
    pass_fwd<NP>(x, tA.w0, tA.w1, tA.w2a, tA.w2b);
    {
        const Tw4 t = load_tw(tw, 0, L);   // in flight during the transpose
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            store_A(X, x[p], L);
            wave_sync();
            load_B_ab(X, x[p], L);
            wave_sync();
        }
        pass_fwd<NP>(x, t.w0, t.w1, t.w2a, t.w2b);
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        store_B_p(X, x[p], L);
        wave_sync();
        load_C(X, x[p], L);
        wave_sync();
    }
}
// the same with the pass-B twiddles supplied by the caller (read from the LDS table)
template <int NP>
__device__ __forceinline__ void fft_fwd_AB_t(Cx (&x)[NP][8], double2 *X, const Tw4 &tA, const Tw4 &t, int L) {
    pass_fwd<NP>(x, tA.w0, tA.w1, tA.w2a, tA.w2b);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        store_A(X, x[p], L);
        wave_sync();
        load_B_ab(X, x[p], L);
        wave_sync();
    }
    pass_fwd<NP>(x, t.w0, t.w1, t.w2a, t.w2b);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        store_B_p(X, x[p], L);
        wave_sync();
        load_C(X, x[p], L);
        wave_sync();
    }
}
template <int NP>
__device__ __forceinline__ void fft_fwd_C(Cx (&x)[NP][8], const Tw4 &tC) {
    pass_fwd<NP>(x, tC.w0, tC.w1, tC.w2a, tC.w2b);
}

// The rounding of the default kernel (round 3): the 1/8 rule without the distance arithmetic.  y = c + 1.5 * 2^50
// has ulp 1/4 while |c| < 2^49, so its low mantissa bits are round(4c): round(4c) = 0 mod 4 iff
// |c - rint(c)| < 1/8 (ties aside), and mantissa bits 2..33 are then rint(c) mod 2^32.  Per
// coefficient: one fp64 add, an alignbit, an and-or into `bad`, the min / max of the high word
// (range: [2^50, 2^51)), instead of round 2's 3 fp64 adds and a max per coefficient (the
// distance itself, with a 1.5 * 2^52 shifter).  Real keys give |c| < 2^48 (the
// product's sigma is 2^44.4); |c| >= 2^49 falls outside the shifter's binade and is flagged.
// tests/test_guard.py emulates these operations.
constexpr uint32_t kQShiftHiLo = 0x43100000u;   // high word of 2^50
constexpr uint32_t kQShiftHiEnd = 0x43200000u;  // high word of 2^51
__device__ __forceinline__ uint32_t torus_of_qchk(double c, uint32_t &bad, uint32_t &hlo, uint32_t &hhi) {
    const double y = c + 0x1.8p50;
    const unsigned long long yb = (unsigned long long)__double_as_longlong(y);
    const uint32_t lo = (uint32_t)yb, hy = (uint32_t)(yb >> 32);
    bad |= lo & 3u;
    hlo = hy < hlo ? hy : hlo;
    hhi = hy > hhi ? hy : hhi;
    return __builtin_amdgcn_alignbit(hy, lo, 2);
}

// high word of a non-negative double: monotone in its value, max-reduced across the wave
__device__ __forceinline__ uint32_t wave_max_hi(double v) {
    uint32_t h = (uint32_t)((unsigned long long)__double_as_longlong(v) >> 32);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)h, off, 64);
        h = o > h ? o : h;
    }
    return h;
}

__device__ __forceinline__ void e6_store(uint32_t *E, int j, uint32_t v, bool third) {
    E[j] = v;
    E[j + kN] = 0u - v;
    if (third) E[j + 2 * kN] = v;
}

// the accumulator polynomial of this wave, coefficient L + 64 r in acc[r], written as its
// periodic negacyclic extension E[k] = +-acc[k mod N] (k < 2240) into the wave's buffer
__device__ __forceinline__ void write_ext(uint32_t *E, const uint32_t (&acc)[16], int L) {
#pragma unroll
    for (int r = 0; r < 16; ++r) e6_store(E, L + 64 * r, acc[r], r < 3);
}

// BK_i rows 2w, 2w + 1 of output c for this lane: 16 x 16 B, all in flight together, as buffer
// loads: the key is one buffer resource (SGPRs), the slice / row / output offset of each row is
// wave-uniform (soffset, SGPR) and the lane's offset loop-invariant (voffset, 2 VGPRs + immediate
// offsets), so a step spends no vector ALU on key addresses (the flat-pointer form recomputed 64-bit
// lane addresses: 12 VALU per wave-step)
__device__ __forceinline__ Cx ld_key_buf(__amdgpu_buffer_rsrc_t rk, int voff, int soff) {
    typedef int i4 __attribute__((ext_vector_type(4)));
    const i4 v = __builtin_bit_cast(i4, __builtin_amdgcn_raw_buffer_load_b128(rk, voff, soff, 0));
    const long long lo = ((long long)(unsigned)v.y << 32) | (unsigned)v.x;
    const long long hi = ((long long)(unsigned)v.w << 32) | (unsigned)v.z;
    return Cx{__longlong_as_double(lo), __longlong_as_double(hi)};
}
// row0 = the key row index (i * 8 + 4 w) of rows (2w, 2w + 1) of slice i, wave-uniform
__device__ __forceinline__ void load_bk(Cx (&b)[2][8], __amdgpu_buffer_rsrc_t rk, int row0, int c, int L) {
    const int s0 = __builtin_amdgcn_readfirstlane((row0 + c) * 512 * 16);
    const int s1 = s0 + 2 * 512 * 16;
    const int v = L * 16;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        b[0][r] = ld_key_buf(rk, v + r * 1024, s0);
        b[1][r] = ld_key_buf(rk, v + r * 1024, s1);
    }
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t key_rsrc(const double2 *bk) {
    // raw buffer of the whole FFT-domain key (32.8 MB), dword 3 = the gfx9 default format
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double2 *>(bk), 0, 0x7fffffff, 0x00020000);
}
// Y = D_0 (x) BK[row 2w][c] + D_1 (x) BK[row 2w + 1][c], layout C
// Y = o + sum_p D_p b_p: the second MAC seeded with the partner wave's partial sum (its first
// products become FMAs and the 16 partial-sum adds disappear)
__device__ __forceinline__ void mac6_seeded(const Cx (&D)[2][8], const Cx (&b)[2][8], const Cx (&o)[8], Cx (&Y)[8]) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const Cx &b0 = b[0][r], &b1 = b[1][r];
        double re = fma_(D[0][r].re, b0.re, o[r].re);
        double im = fma_(D[0][r].re, b0.im, o[r].im);
        re = fma_(-D[0][r].im, b0.im, re);
        im = fma_(D[0][r].im, b0.re, im);
        re = fma_(D[1][r].re, b1.re, re);
        im = fma_(D[1][r].re, b1.im, im);
        re = fma_(-D[1][r].im, b1.im, re);
        im = fma_(D[1][r].im, b1.re, im);
        Y[r] = Cx{re, im};
    }
}
__device__ __forceinline__ void mac6(const Cx (&D)[2][8], const Cx (&b)[2][8], Cx (&Y)[8]) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const Cx &b0 = b[0][r], &b1 = b[1][r];
        double re = D[0][r].re * b0.re;
        double im = D[0][r].re * b0.im;
        re = fma_(-D[0][r].im, b0.im, re);
        im = fma_(D[0][r].im, b0.re, im);
        re = fma_(D[1][r].re, b1.re, re);
        im = fma_(D[1][r].re, b1.im, im);
        re = fma_(-D[1][r].im, b1.im, re);
        im = fma_(D[1][r].im, b1.re, im);
        Y[r] = Cx{re, im};
    }
}


// compact LDS twiddle table (double2 entries): forward pass B [4][8] (by L >> 3), forward pass C
// [4][64], inverse pass B [4][8] (by L & 7), inverse pass A [4][64], post-twist [8][64]
constexpr int kT7FwdB = 0, kT7FwdC = 32, kT7InvB = 288, kT7InvA = 320, kT7Post = 576, kT7Words = 1088;

// source index in the global v6 table (build_v6_twiddles) of compact entry e
__device__ __forceinline__ int t7_src(int e) {
    if (e < kT7FwdC) return 4 + (e >> 3) * 64 + (e & 7) * 8;
    if (e < kT7InvB) return 260 + (e - kT7FwdC);
    if (e < kT7InvA) return kTwInv + ((e - kT7InvB) >> 3) * 64 + ((e - kT7InvB) & 7);
    if (e < kT7Post) return kTwInv + 256 + (e - kT7InvA);
    return kTwPost + (e - kT7Post);
}

// v6's compact table: as above up to inverse pass A, whose first twiddle is a zeta^-L, then the
// lane factor zeta^-L [64] in place of the 8 KB post-twist table
constexpr int kT8Sig = 576, kT8Words = 640;
static_assert(kT8Sig == kT7Post, "v6 and v7 tables agree up to the post-twist");
__device__ __forceinline__ int t8_src(int e) {
    if (e < kT7InvA) return t7_src(e);
    if (e < kT7InvA + 64) return kTwInvAs + (e - kT7InvA);
    if (e < kT8Sig) return kTwInv + 256 + (e - kT7InvA);
    return kTwSig + (e - kT8Sig);
}

__device__ __forceinline__ Tw4 tw7_fwdB(const double2 *t, int L) {
    const double2 *p = t + kT7FwdB + (L >> 3);
    return Tw4{ld(p), ld(p + 8), ld(p + 16), ld(p + 24)};
}
__device__ __forceinline__ Tw4 tw7_fwdC(const double2 *t, int L) {
    const double2 *p = t + kT7FwdC + L;
    return Tw4{ld(p), ld(p + 64), ld(p + 128), ld(p + 192)};
}
__device__ __forceinline__ Tw4 tw7_invB(const double2 *t, int L) {
    const double2 *p = t + kT7InvB + (L & 7);
    return Tw4{ld(p), ld(p + 8), ld(p + 16), ld(p + 24)};
}
__device__ __forceinline__ Tw4 tw7_invA(const double2 *t, int L) {
    const double2 *p = t + kT7InvA + L;
    return Tw4{ld(p), ld(p + 64), ld(p + 128), ld(p + 192)};
}

// The linear combination x = (0, c) + sa X + sb Y + sc Z that feeds one blind rotation (gate
// prologues boot-gates.cu:98-448; a circuit row adds a third input for MAJ / XOR3); y / z may
// be null.
struct RowTerms6 {
    int32_t c, sa, sb, sc;
    const int32_t *xa, *xb, *ya, *yb, *za, *zb;
};

}  // namespace
}  // namespace tfhe_amd
