// fft_wave.h — one wave's share of the fp64 negacyclic FFT external product (v6 blind
// rotation): complex type, butterflies, the three radix-8 register passes and their LDS
// transposes, twiddle tables, the mod-2^32 rounding and the key MAC; the radix-16 forward of the
// opt-in v10.  Design: DESIGN.md §3.1 / §5.4b, emulations: scripts/emu_v6.py, scripts/emu_v10.py.
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
// [1668, 1672) the radix-16 forward's (v10) pass-1 stage-3 twiddles W[3][0, 2, 4, 6] (stages 0..2
// reuse [0, 4)); [1672, 1928) its pass-2 table in the compact order of kT10P2 below
constexpr int kTwR16U = 1668;
constexpr int kTwR16P2 = 1672;

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
// FFT-domain key loads.  A/B variants (cache policy of the key stream, which every ciphertext
// of the launch reads from L2): TFHE_AMD_V6_BK_NT = nontemporal loads (nt: bypass L1)
__device__ __forceinline__ Cx ld_key(const double2 *p) {
#ifdef TFHE_AMD_V6_BK_NT
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v *>(p));
    return Cx{v.x, v.y};
#else
    return ld(p);
#endif
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
// the same with the pass-B twiddles supplied by the caller (v7: read from LDS)
template <int NP>
__device__ __forceinline__ void fft_fwd_AB_t(Cx (&x)[NP][8], double2 *X, const Tw4 &tA, const Tw4 &t, int L) {
    pass_fwd<NP>(x, tA.w0, tA.w1, tA.w2a, tA.w2b);
#if defined(TFHE_AMD_DIAG_PERMFWD)
    // timing diagnostic (wrong results): the forward A -> B transpose replaced by the cross-lane
    // work a radix-16 forward would need instead (2 x 32 v_permlane{16,32}_swap on the doubles
    // + 16 on the digit words), to price that design before building it
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int r = 0; r < 8; r += 2) {
            unsigned *a = reinterpret_cast<unsigned *>(&x[p][r]);
            unsigned *b = reinterpret_cast<unsigned *>(&x[p][r + 1]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                auto s16 = __builtin_amdgcn_permlane16_swap(a[k], b[k], false, false);
                auto s32 = __builtin_amdgcn_permlane32_swap(s16[0], s16[1], false, false);
                a[k] = s32[0];
                b[k] = s32[1];
            }
            if (r < 4) {
                auto s = __builtin_amdgcn_permlane32_swap(a[0], b[2], false, false);
                a[0] = s[0];
                b[2] = s[1];
            }
        }
#elif !defined(TFHE_AMD_DIAG_NOTRAB) && !defined(TFHE_AMD_DIAG_FWDNOTR)
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        store_A(X, x[p], L);
        wave_sync();
        load_B_ab(X, x[p], L);
        wave_sync();
    }
#endif
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

// rint(c) mod 2^32 for |c| < 2^82 (c within 1/2 of an integer): k = c rounded to a multiple
// of 2^32 by the 1.5*2^84 shifter, then c - k + 1.5*2^52 rounds c - k to an integer in the
// low mantissa word.  All three operations are exact except the final rounding.
__device__ __forceinline__ uint32_t torus_of(double c) {
    constexpr double M1 = 0x1.8p84, M12 = 0x1.8p84 + 0x1.8p52;
    const double s = c + M1;
    const double t = s - M12;
    const double y = c - t;
    return (uint32_t)__double_as_longlong(y);
}

// rint(c) mod 2^32 with the exactness guard's measurement, in one shifter: y = c + 1.5 * 2^52.
// For |c| < 2^51, y lies in [2^52, 2^53) (ulp 1), so y rounds c to the nearest integer and the
// low mantissa word is rint(c) mod 2^32; q = y - 1.5 * 2^52 and c - q are exact, and
// mx = max(mx, |c - q|) is the rounding distance.  Outside that range (the product bound is
// |c| <= 2^52; real keys give < 2^48) y's exponent differs and its low word is not rint(c):
// the high word of y, tracked as hlo = min and hhi = max, must stay in [0x43300000, 0x43400000)
// or the kernel flags the ciphertext (tests/test_guard.py emulates exactly these operations).
// 3 fp64 adds, one fp64 max and two integer min / max per coefficient (the previous form: two
// shifters plus a Fast2Sum error, 5 fp64 ops and a max).  TFHE_AMD_V6_NOGUARD: the shifter
// alone (A/B builds; exact only while |c| < 2^51).
constexpr uint32_t kShiftHiLo = 0x43300000u;   // high word of 2^52
constexpr uint32_t kShiftHiEnd = 0x43400000u;  // high word of 2^53
__device__ __forceinline__ uint32_t torus_of_chk(double c, double &mx, uint32_t &hlo, uint32_t &hhi) {
    constexpr double M2 = 0x1.8p52;
    const double y = c + M2;
#ifndef TFHE_AMD_V6_NOGUARD
    const double q = y - M2;
    mx = __builtin_fmax(mx, __builtin_fabs(c - q));
    const uint32_t hy = (uint32_t)((unsigned long long)__double_as_longlong(y) >> 32);
    hlo = hy < hlo ? hy : hlo;
    hhi = hy > hhi ? hy : hhi;
#endif
    return (uint32_t)__double_as_longlong(y);
}

// The rounding of the default kernel (round 3): the 1/8 rule without the distance arithmetic.  y = c + 1.5 * 2^50
// has ulp 1/4 while |c| < 2^49, so its low mantissa bits are round(4c): round(4c) = 0 mod 4 iff
// |c - rint(c)| < 1/8 (ties aside), and mantissa bits 2..33 are then rint(c) mod 2^32.  Per
// coefficient: one fp64 add, an alignbit, an and-or into `bad`, the min / max of the high word
// (range: [2^50, 2^51)), instead of 3 fp64 adds and a max (torus_of_chk above, kept for the
// experimental v8 and the TFHE_AMD_V6_DISTGUARD A/B build).  Real keys give |c| < 2^48 (the
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

// BK_i rows 2w, 2w + 1 of output c for this lane: 16 x 16 B, all in flight together
__device__ __forceinline__ void load_bk(Cx (&b)[2][8], const double2 *bk, int c) {
#ifdef TFHE_AMD_DIAG_NOBK
    // timing diagnostic only (wrong results): no key traffic
    const double s = 1e-9 * (double)(int)(reinterpret_cast<uintptr_t>(bk) & 0xffff);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        b[0][r] = Cx{s + r, s - c};
        b[1][r] = Cx{s - r, s + c};
    }
    return;
#endif
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        b[0][r] = ld_key(bk + c * 512 + r * 64);
        b[1][r] = ld_key(bk + (2 + c) * 512 + r * 64);
    }
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

// ---- the radix-16 forward (v10; scripts/emu_v10.py emulates exactly this data flow)
// compact LDS table: entries [0, 256) = the pass-2 table (per-lane twiddles, by m = L & 15 or
// t = L & 31): t4[m] (16), t5[m] (16), t6[q][m] (2 x 16), t7[q][m] (4 x 16), t8[q][t] (4 x 32);
// [256, 288) unused; from kT7InvB on the v6 compact table (the inverse is v6's)
constexpr int kT10P2 = 0, kT10T5 = 16, kT10T6 = 32, kT10T7 = 64, kT10T8 = 128, kT10P2Words = 256;
static_assert(kT10P2Words <= kT7FwdC + 256, "the pass-2 table replaces the forward passes B / C entries");
__device__ __forceinline__ int t10_src(int e) {
    if (e < kT10P2Words) return kTwR16P2 + e;
    if (e < kT7InvB) return 0;
    return t8_src(e);
}
// 64-bit halves exchanged by the cross-lane swaps, one dword at a time
__device__ __forceinline__ void swap32_cx(Cx &a, Cx &b) {   // v_permlane32_swap vdst = a, src = b
    const unsigned long long ar = __double_as_longlong(a.re), ai = __double_as_longlong(a.im);
    const unsigned long long br = __double_as_longlong(b.re), bi = __double_as_longlong(b.im);
    auto s0 = __builtin_amdgcn_permlane32_swap((unsigned)ar, (unsigned)br, false, false);
    auto s1 = __builtin_amdgcn_permlane32_swap((unsigned)(ar >> 32), (unsigned)(br >> 32), false, false);
    auto s2 = __builtin_amdgcn_permlane32_swap((unsigned)ai, (unsigned)bi, false, false);
    auto s3 = __builtin_amdgcn_permlane32_swap((unsigned)(ai >> 32), (unsigned)(bi >> 32), false, false);
    a.re = __longlong_as_double((long long)(((unsigned long long)s1[0] << 32) | s0[0]));
    b.re = __longlong_as_double((long long)(((unsigned long long)s1[1] << 32) | s0[1]));
    a.im = __longlong_as_double((long long)(((unsigned long long)s3[0] << 32) | s2[0]));
    b.im = __longlong_as_double((long long)(((unsigned long long)s3[1] << 32) | s2[1]));
}
__device__ __forceinline__ void swap16_cx(Cx &a, Cx &b) {   // v_permlane16_swap vdst = a, src = b
    const unsigned long long ar = __double_as_longlong(a.re), ai = __double_as_longlong(a.im);
    const unsigned long long br = __double_as_longlong(b.re), bi = __double_as_longlong(b.im);
    auto s0 = __builtin_amdgcn_permlane16_swap((unsigned)ar, (unsigned)br, false, false);
    auto s1 = __builtin_amdgcn_permlane16_swap((unsigned)(ar >> 32), (unsigned)(br >> 32), false, false);
    auto s2 = __builtin_amdgcn_permlane16_swap((unsigned)ai, (unsigned)bi, false, false);
    auto s3 = __builtin_amdgcn_permlane16_swap((unsigned)(ai >> 32), (unsigned)(bi >> 32), false, false);
    a.re = __longlong_as_double((long long)(((unsigned long long)s1[0] << 32) | s0[0]));
    b.re = __longlong_as_double((long long)(((unsigned long long)s1[1] << 32) | s0[1]));
    a.im = __longlong_as_double((long long)(((unsigned long long)s3[0] << 32) | s2[0]));
    b.im = __longlong_as_double((long long)(((unsigned long long)s3[1] << 32) | s2[1]));
}
// The forward's transpose buffer: per half (digit polynomial) 512 positions at slot n + (n >> 5),
// conflict-free with the register index in the immediate offset on both sides
constexpr int kR16Half = 528, kR16Slots = 2 * kR16Half;
// The lane that holds slot 8 L' + r of layout C after the radix-16 forward
__device__ __forceinline__ int r16_lane(int L) { return (L >> 5) + 2 * ((L >> 4) & 1) + 4 * (L & 15); }
// Pass 1 and the transpose.  HI / LO: the digits of coefficients L + 64 r of this wave's
// accumulator polynomial (r < 16).  The halves split by digit: after one v_permlane32_swap per
// register the lower lanes hold the high digits of coefficients l + 64 r (HI) and l + 32 + 64 r (LO),
// the upper lanes the low digits, l = L & 31; so position n = l + 32 r' of the lane's digit
// polynomial (z_n = a_n + i a_{n + 512}) is Z[2 k] = HI[k] + i HI[k + 8], Z[2 k + 1] = LO[k] +
// i LO[k + 8].  Pass 1 = stages 0..3 (n bits 8..5 = r' bits 3..0, uniform twiddles: u[0..3] as
// v6's pass A, u3[0..3] = W[3][0, 2, 4, 6]); then ONE transpose through X (both halves,
// kR16Slots) to lane (m, b') = (L & 15, (L >> 4) & 1) holding
// n = b' + 2 r'' + 32 m.
__device__ __forceinline__ void r16_pass1_transpose(const int32_t (&HI)[16], const int32_t (&LO)[16], Cx (&Z)[16],
                                                    double2 *X, const Tw4 &u, const Tw4 &u3, int L) {
    int32_t E[16], O[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        auto s = __builtin_amdgcn_permlane32_swap((unsigned)HI[r], (unsigned)LO[r], false, false);
        E[r] = (int32_t)s[0];
        O[r] = (int32_t)s[1];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        Z[2 * k] = Cx{(double)E[k], (double)E[k + 8]};
        Z[2 * k + 1] = Cx{(double)O[k], (double)O[k + 8]};
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) bf_fwd<false>(Z[r], Z[r + 8], u.w0);                 // stage 0 (bit 8)
#pragma unroll
    for (int r = 0; r < 4; ++r) {                                                        // stage 1 (bit 7)
        bf_fwd<false>(Z[r], Z[r + 4], u.w1);
        bf_fwd<true>(Z[r + 8], Z[r + 12], u.w1);
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {                                                        // stage 2 (bit 6)
        const Cx &t = b < 2 ? u.w2a : u.w2b;
        const int r0 = 4 * b;
        if (b & 1) {
            bf_fwd<true>(Z[r0], Z[r0 + 2], t);
            bf_fwd<true>(Z[r0 + 1], Z[r0 + 3], t);
        } else {
            bf_fwd<false>(Z[r0], Z[r0 + 2], t);
            bf_fwd<false>(Z[r0 + 1], Z[r0 + 3], t);
        }
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {                                                        // stage 3 (bit 5)
        const Cx &t = (b >> 1) == 0 ? u3.w0 : (b >> 1) == 1 ? u3.w1 : (b >> 1) == 2 ? u3.w2a : u3.w2b;
        if (b & 1) bf_fwd<true>(Z[2 * b], Z[2 * b + 1], t);
        else bf_fwd<false>(Z[2 * b], Z[2 * b + 1], t);
    }
    double2 *Xh = X + (L >> 5) * kR16Half;
    const int l = L & 31;
#pragma unroll
    for (int r = 0; r < 16; ++r) st(Xh + l + 33 * r, Z[r]);
    wave_sync();
    const int m = L & 15, b1 = (L >> 4) & 1;
#pragma unroll
    for (int r = 0; r < 16; ++r) Z[r] = ld(Xh + b1 + 33 * m + 2 * r);
    wave_sync();
}
// Pass 2 = stages 4..7 (n bits 4..1 = r'' bits 3..0; per-lane twiddles from the compact table),
// stage 8 (bit 0 = lane bit 4) through v_permlane16_swap, then the two digits' spectra re-paired
// in every lane by v_permlane32_swap: D[d][r] = digit d at slot 8 r16_lane(L) + r (layout C)
__device__ __forceinline__ void r16_pass2(Cx (&Z)[16], Cx (&D)[2][8], const double2 *shtw, int L) {
    const int m = L & 15, t = L & 31;
    {
        const Cx t4 = ld(shtw + kT10P2 + m);
#pragma unroll
        for (int r = 0; r < 8; ++r) bf_fwd<false>(Z[r], Z[r + 8], t4);                 // stage 4
    }
    {
        const Cx t5 = ld(shtw + kT10T5 + m);
#pragma unroll
        for (int r = 0; r < 4; ++r) {                                                    // stage 5
            bf_fwd<false>(Z[r], Z[r + 4], t5);
            bf_fwd<true>(Z[r + 8], Z[r + 12], t5);
        }
    }
    {
        const Cx t6a = ld(shtw + kT10T6 + m), t6b = ld(shtw + kT10T6 + 16 + m);
#pragma unroll
        for (int b = 0; b < 4; ++b) {                                                    // stage 6
            const Cx &tw = b < 2 ? t6a : t6b;
            const int r0 = 4 * b;
            if (b & 1) {
                bf_fwd<true>(Z[r0], Z[r0 + 2], tw);
                bf_fwd<true>(Z[r0 + 1], Z[r0 + 3], tw);
            } else {
                bf_fwd<false>(Z[r0], Z[r0 + 2], tw);
                bf_fwd<false>(Z[r0 + 1], Z[r0 + 3], tw);
            }
        }
    }
    {
        Cx t7[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) t7[q] = ld(shtw + kT10T7 + 16 * q + m);
#pragma unroll
        for (int b = 0; b < 8; ++b) {                                                    // stage 7
            if (b & 1) bf_fwd<true>(Z[2 * b], Z[2 * b + 1], t7[b >> 1]);
            else bf_fwd<false>(Z[2 * b], Z[2 * b + 1], t7[b >> 1]);
        }
    }
    {
        Cx t8[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) t8[q] = ld(shtw + kT10T8 + 32 * q + t);
#pragma unroll
        for (int p = 0; p < 8; ++p) swap16_cx(Z[p], Z[p + 8]);                          // stage 8
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            if (p & 1) bf_fwd<true>(Z[p], Z[p + 8], t8[p >> 1]);
            else bf_fwd<false>(Z[p], Z[p + 8], t8[p >> 1]);
        }
    }
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            swap32_cx(Z[p + 8 * e], Z[p + 4 + 8 * e]);
            D[0][e + 2 * p] = Z[p + 8 * e];
            D[1][e + 2 * p] = Z[p + 4 + 8 * e];
        }
}
// The inverse's C -> B transpose from the radix-16 forward's lane order: position n (k = n >> 3,
// j = n & 7) at slot 16 k + (j ^ t(k >> 2)), t = bits 1 and 3 of its argument exchanged.  Conflict
// free both ways: a store group of 16 lanes holds k >> 2 = L & 15 (all 16 values of t), a load
// group two k's 8 apart (t differs in bit 3).  1024 slots (v10).
__device__ __forceinline__ int r16_t(int m) { return (m & 5) | ((m >> 2) & 2) | ((m & 2) << 2); }
__device__ __forceinline__ void store_C16(double2 *X, const Cx (&x)[8], int Lp) {
    const int a = 16 * Lp + r16_t(Lp >> 2);
#pragma unroll
    for (int r = 0; r < 8; ++r) st(X + (a ^ r), x[r]);
}
__device__ __forceinline__ void load_B16(const double2 *X, Cx (&x)[8], int L) {
    const int h = L >> 3;
    const int b0 = 128 * h + ((L & 7) ^ r16_t(2 * h)), b1 = b0 ^ 1;
#pragma unroll
    for (int r = 0; r < 8; ++r) x[r] = ld(X + (r < 4 ? b0 : b1) + 16 * r);
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
