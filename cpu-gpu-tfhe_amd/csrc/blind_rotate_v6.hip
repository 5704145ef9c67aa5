// blind_rotate_v6.hip — blind rotation with an fp64 negacyclic FFT external product.
//
// The reference computes tGswFFTExternMulToTLwe with a double-precision FFT
// (tgsw-fft-operations.cu:124-264: IntPolynomial_ifft of the decomposition, the
// LagrangeHalfCPolynomial MAC with the FFT-domain key, TorusPolynomial_fft back).  v1..v5 use an
// exact 2-prime NTT instead; on CDNA4 that costs ~22 VALU issue cycles per radix-2 butterfly
// per prime, where the fp64 butterfly below costs 6 full-rate v_fma_f64 (MI355X: fp64 vector
// FMA at the fp32 rate), so v6 returns to the reference's arithmetic, MI355X-shaped:
//
//  * one ciphertext = 2 waves (128 threads); wave w owns accumulator polynomial w (16 Torus32
//    coefficients per lane, in registers), decomposes it into its 2 digit polynomials (rows 2w,
//    2w+1 of the TGSW key), runs 2 forward transforms, MACs them with BK_i rows (2w, 2w+1) for
//    BOTH output polynomials, hands the partial sum of output 1-w to the other wave through LDS,
//    and runs one inverse transform for output w;
//  * transform = 512-point complex FFT of the folded polynomial z_n = a_n + i a_{n+512}
//    evaluated at the 512 roots of X^512 = i (those are roots of X^1024 + 1, so products are
//    negacyclic): Cooley-Tukey with the twist merged into the twiddles, three radix-8 register
//    passes (layouts A, B, C: 8 complex per lane) joined by two LDS transposes.  Its output is
//    in bit-reversed order of zeta omega^k, so the inverse is a radix-2 DIT on that order
//    (constant twiddles in pass C, per-lane ones in passes B and A) plus a zeta^-n post-twist;
//    the 1/512 scale is folded into the key.  scripts/emu_v6.py emulates this exact data flow.
//  * rounding: |coefficient| < 2^52 and the FFT error stays below ~0.05 (emu_v6.py: 0.045 worst
//    on random keys) << 1/2, so rint() of the result equals the exact product, i.e. the same
//    integers the exact NTT kernels produce; the mod-2^32 reduction is 3 exact fp64 operations.
//  * each wave has ONE 9 KB LDS buffer: per step it holds the periodic negacyclic extension
//    E[k] = +-acc[k mod N] (k < 2240: the rotation X^a reads E[(j - a) mod 2N] with one base per
//    quarter of the lane's coefficients; launches above one workgroup per CU rotate in registers
//    with ds_bpermute instead, cmux_v6 RREG), then the FFT transposes, then the partial sum
//    handed to the other wave; the per-lane twiddles are read from a 10 KB LDS copy (29.7 KB per
//    ciphertext, 4 workgroups per CU), so the key is the only global load in the loop.
//  * issue priority is steered per launch (set_prio_level): a rotation phased by the workgroup's
//    rank on its CU for the one-round launches a batch is split into (by step if the split is
//    disabled).
//  * round 5's radix-16 generation (v10 / v10s: one LDS transpose per forward transform pair,
//    cross-lane swaps for the rest) was exact and measured neutral at the throughput batches and
//    slower below; it was removed in round 6 (profiles/r05i_*, r05k_*).
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <vector>
#include "engine.h"
#include "modarith.h"
#include "fft_wave.h"

namespace tfhe_amd {

namespace {

constexpr int kV6Threads = 128;
// Register budget: 2 waves per SIMD (256 VGPRs; 16 key loads in flight).  A 1024-ciphertext
// launch has exactly 2 waves per SIMD, and 3- or 4-wave budgets (8 loads in flight, <= 168 or
// 128 VGPRs) measured slower at every batch size (B = 2048: 8.4 -> 16.6 ms).
constexpr int kV6Waves = 2;

#ifdef TFHE_AMD_V6_STAMPS
// phase timing diagnostics: shader-clock cycles per phase, accumulated in (uniform) registers
// and written by waves 0 and 1 of workgroup 0 at the end; read with tfhe_amd_debug_v6_stamps
// (scripts/v6_stamps.py)
__device__ unsigned long long g_v6_stamps[2][12];
struct V6Stamps {
    unsigned long long acc[10] = {0};
    unsigned long long prev = 0;
};
#define V6_STAMP(k)                                                 \
    do {                                                             \
        const unsigned long long now = __builtin_amdgcn_s_memtime(); \
        stamps.acc[k] += now - stamps.prev;                          \
        stamps.prev = now;                                           \
    } while (0)
// per-workgroup wall-clock window and placement: [start_rt, end_rt, start_clk, end_clk, hw_id, xcc_id]
// (s_memrealtime: constant 100 MHz; s_memtime: shader clock), read with tfhe_amd_debug_v6_wgtime
constexpr int kWgSlots = 8192;
__device__ unsigned long long g_v6_wg[kWgSlots][6];
__device__ __forceinline__ unsigned int hwreg_hw_id() {
    unsigned int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
    return v;
}
__device__ __forceinline__ unsigned int hwreg_xcc_id() {
    unsigned int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v;
}
#define V6_STAMPS_PARAM , V6Stamps &stamps
#define V6_STAMPS_ARG , stamps
#else
#define V6_STAMP(k) do {} while (0)
#define V6_STAMPS_PARAM
#define V6_STAMPS_ARG
#endif

// issue-order fence for the LDS read groups of the inverse
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

struct __attribute__((aligned(16))) V6Ct {   // one ciphertext's LDS
    double2 X[2][kXSlots];           // per-wave buffer (9 KB): accumulator extension, FFT transposes, partial sums
    short bara[512];                 // rotation amounts < 2N (16 bit: 8 workgroups fit a CU)
    int barb;
    int sync[2];                     // PS: the steps each wave has handed its partial sum over for
};
template <int C>
struct __attribute__((aligned(16))) V6SharedC {
    V6Ct ct[C];                      // C ciphertexts per workgroup share ...
    double2 tw[kT8Words];            // ... the per-lane twiddles (compact table, fft_wave.h)
};
using V6Shared = V6SharedC<1>;
static_assert(kExt6 * 4 <= kXSlots * 16, "accumulator extension fits the wave buffer");

struct V6Args {
    const double2 *bk;   // [kn][4 rows][2 c][8 r][64 L]: FFT-domain key / 512, slot 8 L + r
    uint32_t *flags;     // exactness guard (engine.h Guard): [2 slot + w] max rounding distance, or null
    uint32_t *stats;     // [1]: the largest distance (high word) seen
    const double2 *tw;   // build_v6_twiddles' table; copied to LDS in compact form (fft_wave.h)
    int prio;            // issue-priority policy, see set_prio_level
    int prio_shift;      // policy 5: steps per level = 2^prio_shift
    int cus;             // compute units (workgroup b shares its CU with b +- cus, b +- 2 cus, ...)
};

// Issue priority.  A SIMD holds two waves (different workgroups) and the hardware arbitrates
// between them by priority, then age, so by default the oldest workgroup of a CU runs ahead and
// the youngest trails (B = 1024: 2.7 ms vs 3.9 ms per workgroup, scripts/v6_wgtime.py), and
// the launch lasts as long as the slowest.  Workgroup b shares its CU with b +- CUs, b +- 2 CUs,
// b +- 3 CUs (dispatch order; ranks 0/1 and 2/3 share SIMD pairs).  Policy 5 (one round of
// workgroups, the default): every 8 steps each workgroup moves one level up (mod 4) from a start
// level 2 x rank, so SIMD partners always sit two levels apart and trade first place every 16
// steps (B = 1024: 3.56 ms with no policy -> 3.21; the same rotation from a hashed start level:
// 3.36).  Policy 1 (more workgroups than fit at once): priority 3 - i / 128 by step, so
// workgroups dispatched later, still early in their 500 steps, go first (B = 4096 in one launch:
// 15.4 -> 13.7 ms).  Policy 0: hardware default (the paired kernel).
__device__ __forceinline__ void set_prio_level(unsigned lvl) {
    switch (lvl & 3) {
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
}


// one CMux step, wave w: acc_w += [(X^a - 1) ACC] (x) BK_i, output polynomial w.  The
// accumulator lives in registers; the wave's LDS buffer holds, in turn, its periodic extension
// (rotation reads), the FFT transposes and the partial sum handed to the other wave.
// PS (the paired kernel, two ciphertexts per workgroup, the default there): the two waves of a
// ciphertext meet through LDS step counters instead of the workgroup barrier, so that the
// workgroup's two ciphertexts are not held in lock-step.  With one wave per SIMD nothing hides a
// wave's LDS round trips; in lock-step the four waves of a CU issued their transposes together and
// queued behind each other on the CU's LDS, out of step they interleave (B = 512: -12 %).
template <int WAVES, bool RREG, bool RSW = false, bool PS = false>
__device__ __forceinline__ void cmux_v6(V6Ct &sh, const double2 *shtw, const V6Args &g, const Tw4 &tA,
                                        int i, int a, int w, int &own,
                                        int L, uint32_t (&acc)[16], double &mx, uint32_t &hlo, uint32_t &hhi,
                                        uint32_t &bad, int &seq V6_STAMPS_PARAM) {
    double2 *X = sh.X[own];
    uint32_t *E = reinterpret_cast<uint32_t *>(X);
    V6_STAMP(9);
    const __amdgpu_buffer_rsrc_t rk = key_rsrc(g.bk);
    const int row0 = i * 8 + w * 4;   // rows (2w, 2w + 1) of slice i, wave-uniform
    Cx bv[2][8];                  // 16 key loads in flight (256-VGPR budget: 2 waves per SIMD)
    // (X^a - 1) ACC_w and its signed gadget digits (tgsw-functions.cu:300-413):
    // hi = sext10 bits 22..31 of diff + off + 2^31, lo = sext10 bits 12..21 of diff + off + 2^21
    Cx D[2][8];
    auto digits = [&](int r, uint32_t rot) {
        const uint32_t diff = rot - acc[r];
        const int32_t hi = (int32_t)(diff + (kDecompOffset + 0x80000000u)) >> 22;
        const int32_t lo = __builtin_amdgcn_sbfe((int32_t)(diff + (kDecompOffset + 0x200000u)), 12, 10);
        if (r < 8) {
            D[0][r].re = (double)hi;
            D[1][r].re = (double)lo;
        } else {
            D[0][r - 8].im = (double)hi;
            D[1][r - 8].im = (double)lo;
        }
    };
    if constexpr (RREG) {
        // X^a ACC_w without the LDS extension: coefficient j = L + 64 r needs (j - a) mod 2N; with
        // a = 64 q + s, lane L takes lane (L - s) mod 64's register r - q (r - q - 1 for L < s)
        // of the negacyclic ring of 32 registers (16 held, the other 16 their negatives): one
        // ds_bpermute per register, then a rotation by the wave-uniform q in 5 binary stages.
        // Used for launches of more than one workgroup per CU (B = 512 / 1024 / 4096: -1.0 /
        // -0.8 / -0.7 %); the LDS extension stays for the latency case (B = 1: 1.68 vs 1.70 ms).
        (void)E;
        const int aa = __builtin_amdgcn_readfirstlane(a) & (k2N - 1);
        const int s = aa & 63, q = aa >> 6;
        const int src = ((L - s) & 63) << 2;
        uint32_t V[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) V[r] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)acc[r]);
        const bool lo = L < s;
        if constexpr (RSW) {
            // RSW (the one-ciphertext-per-workgroup kernels of launches above 2 ciphertexts per
            // CU, i.e. the throughput launches): one of 32 static register permutations chosen by a
            // scalar branch tree on q, with the lane select L < s folded into each case, so every
            // case writes the 16 digit sources straight from V: 16 selects plus its negations
            // instead of up to 5 conditional stages of 16 (B = 1 024 / 4 096 -0.5 / -0.35 %
            // against the stages, profiles/r03_rswitch_ab.txt; the fold another -1.2 / -1.1 %,
            // profiles/r06m_rswitch_select_ab.txt).  At B = 512, one wave per SIMD, the branch tree
            // on the critical path cost +1 %, and with the fold it is neutral (profiles/r06n_*),
            // so the paired kernel keeps the stages.
            uint32_t O[16];
            // register k of the negacyclic ring of 32 (k in [-32, 16)): V, or its negation below 0
            auto ring = [&](int k) -> uint32_t { return k >= 0 ? V[k] : (k >= -16 ? 0u - V[k + 16] : V[k + 32]); };
            switch (q) {
#define V6_SEL_CASE(Q)                                                                            \
    case Q: {                                                                                     \
        _Pragma("unroll") for (int r = 0; r < 16; ++r)                                            \
            O[r] = lo ? (r ? ring(r - 1 - (Q)) : 0u - ring(15 - (Q))) : ring(r - (Q));            \
    } break;
                V6_SEL_CASE(0) V6_SEL_CASE(1) V6_SEL_CASE(2) V6_SEL_CASE(3) V6_SEL_CASE(4) V6_SEL_CASE(5)
                V6_SEL_CASE(6) V6_SEL_CASE(7) V6_SEL_CASE(8) V6_SEL_CASE(9) V6_SEL_CASE(10) V6_SEL_CASE(11)
                V6_SEL_CASE(12) V6_SEL_CASE(13) V6_SEL_CASE(14) V6_SEL_CASE(15) V6_SEL_CASE(16) V6_SEL_CASE(17)
                V6_SEL_CASE(18) V6_SEL_CASE(19) V6_SEL_CASE(20) V6_SEL_CASE(21) V6_SEL_CASE(22) V6_SEL_CASE(23)
                V6_SEL_CASE(24) V6_SEL_CASE(25) V6_SEL_CASE(26) V6_SEL_CASE(27) V6_SEL_CASE(28) V6_SEL_CASE(29)
                V6_SEL_CASE(30)
                default: V6_SEL_CASE(31)
#undef V6_SEL_CASE
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) digits(r, O[r]);
        } else {
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
#pragma unroll
            for (int r = 0; r < 16; ++r) digits(r, lo ? (r ? V[r - 1] : 0u - V[15]) : V[r]);
        }
    } else {
        write_ext(E, acc, L);
        wave_sync();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int base = (L + 256 * q - a) & (k2N - 1);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) digits(4 * q + rr, E[base + 64 * rr]);
        }
    }
    wave_sync();
    V6_STAMP(0);
    fft_fwd_AB_t<2>(D, X, tA, tw7_fwdB(shtw, L), L);
    V6_STAMP(1);
    // MAC with rows 2w + p of BK_i ([p][c][r][L], slot 8 L + r): output 1 - w first, handed
    // to the other wave through this wave's buffer, then output w.  The first key slice is in
    // flight during pass C, the second during the first MAC, the hand-over and the barrier.
    Cx Y[8];
    // (issuing them at the top of the step instead, in flight for the whole forward transform,
    // measured no faster: B = 1 1.69 -> 1.75 ms, B = 1024 / 4096 unchanged)
    // (a one-wave build of the paired kernel that loads each key slice a whole step ahead, 64 more
    // VGPRs live across the step, measured slower: B = 512 2.336 vs 2.273 ms, profiles/r04f_*)
    {
        const Tw4 tC = tw7_fwdC(shtw, L);
        load_bk(bv, rk, row0, 1 - w, L);
        __builtin_amdgcn_sched_barrier(0);   // keep the 16 loads issued ahead of pass C
        fft_fwd_C<2>(D, tC);
    }
    mac6(D, bv, Y);
    V6_STAMP(2);
    load_bk(bv, rk, row0, w, L);
    __builtin_amdgcn_sched_barrier(0);
    store_C(X, Y, L);
    // the second MAC runs after the barrier and the partner-partial loads, so that its key
    // loads land during those waits (B = 1: 1.69 -> 1.65 ms, B = 1024: -1 %)
    V6_STAMP(3);
    if constexpr (PS) {
        // release: this wave's partial sum (and everything before it in LDS) before its counter
        seq += 1;
        __hip_atomic_store(&sh.sync[w], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        for (int spins = 0;; ++spins) {
            const int v = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&sh.sync[1 - w], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (v >= seq) break;
            if (spins > (1 << 24)) {   // never expected; no hang: the guard's exact kernel recomputes it
                bad = 1u;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    } else {
        (void)seq;
        lds_barrier6();
    }
    V6_STAMP(4);
    // Inverse.  Every LDS read group is issued whole before the arithmetic that consumes it
    // (sched_barrier): at this register budget the scheduler otherwise sinks each ds_read to its use and
    // waits lgkmcnt(0) per pair, or per post-twist twiddle, i.e. one LDS round trip each.
    {
        Cx o[8];
        load_C(sh.X[1 - own], o, L);
        SCHED_FENCE();
        // the partner's partial sum seeds the second MAC (16 fp64 fewer per wave-step: B = 1 / 256
        // / 512 / 1 024 / 4 096 -0.9 / -1.2 / -0.9 / -0.8 / -0.6 %, profiles/r03_seed_mac2_ab.txt,
        // r03_seed_mac2_latency_ab.txt)
        mac6_seeded(D, bv, o, Y);
    }
    pass_dit_C(Y);
    const Tw4 tB = tw7_invB(shtw, L);
    V6_STAMP(5);
    // Buffer hand-over instead of a second barrier: the wave goes on in the partner's buffer,
    // which the partner has finished with (it wrote its partial sum there before the barrier and
    // now works in ours); LDS runs this wave's reads of it before its stores.  The two waves swap
    // buffers every step (B = 1024: one s_barrier per step instead of two).
    X = sh.X[1 - own];
    own = 1 - own;
    V6_STAMP(6);
    store_C(X, Y, L);
    wave_sync();
    load_B_p(X, Y, L);
    SCHED_FENCE();
    pass_dit(Y, tB.w0, tB.w1, tB.w2a, tB.w2b);
    {
        // post-twist zeta^-n, n = L + 64 r = zeta^-L (lane) x e^{-2 pi i r / 32} (register): the
        // lane factor scales the pass's inputs — the u inputs of its first butterflies here, the v
        // inputs through its first twiddle, stored as a zeta^-L — and the register factor its
        // outputs, from constants: 11 complex products and one twiddle load instead of 8 and 8
        // (B = 1024: the 8 post-twist loads alone cost 1.3 %)
        const Tw4 tI = tw7_invA(shtw, L);
        const Cx sg = ld(shtw + kT8Sig + L);
        wave_sync();
        store_B_ab(X, Y, L);
        wave_sync();
        load_A(X, Y, L);
        SCHED_FENCE();
#pragma unroll
        for (int r = 0; r < 8; r += 2) Y[r] = cmul(Y[r], sg);
        pass_dit(Y, tI.w0, tI.w1, tI.w2a, tI.w2b);
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
        for (int r = 1; r < 8; ++r) Y[r] = cmul(Y[r], Cx{kOm[r][0], kOm[r][1]});
    }
    V6_STAMP(7);
    // acc_w += rint(result): coefficient L + 64 r (re) and L + 64 (r + 8) (im); mx tracks the
    // rounding distance for the exactness guard
    // the 1/8 rule on every coefficient through the quarter-ulp shifter (bad, fft_wave.h
    // torus_of_qchk: B = 1 024 / 4 096 -0.9 / -1.1 %, profiles/r03_qguard_ab.txt); the distance
    // itself on one coefficient per lane and step, for the statistic (tfhe_amd_guard_stats; sampling
    // it every fourth step instead saves 3 fp64 per wave-step only with a real branch, which splits
    // the inverse's tail from the rounding)
    mx = __builtin_fmax(mx, __builtin_fabs(Y[0].re - __builtin_rint(Y[0].re)));
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        acc[r] += torus_of_qchk(Y[r].re, bad, hlo, hhi);
        acc[r + 8] += torus_of_qchk(Y[r].im, bad, hlo, hhi);
    }
    wave_sync();
    V6_STAMP(8);
}

// C ciphertexts per workgroup (128 C threads; ciphertext threadIdx.x / 128 uses sh): with C = 2
// the workgroup's barriers lock-step both, so neither skips a_i = 0 steps (the identity CMux is
// exact: zero digits, zero transforms, zero products).  live = false: a padding ciphertext that
// computes but writes nothing.
template <int WAVES, bool RREG, int C = 1, bool PS = false>
__device__ __forceinline__ void br_v6_body(V6Ct &sh, double2 *shtw, const V6Args &g, const RowTerms6 &t, int32_t mu,
                                           int32_t *__restrict__ ua, int32_t *__restrict__ ub, size_t slot,
                                           bool live = true) {
    const int tid = threadIdx.x & (kV6Threads - 1);
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = tid & 63;
#ifdef TFHE_AMD_V6_STAMPS
    const int wg = blockIdx.x + blockIdx.y * gridDim.x;
    if (tid == 0 && wg < kWgSlots) {
        g_v6_wg[wg][0] = __builtin_amdgcn_s_memrealtime();
        g_v6_wg[wg][2] = __builtin_amdgcn_s_memtime();
        g_v6_wg[wg][4] = hwreg_hw_id();
        g_v6_wg[wg][5] = hwreg_xcc_id();
    }
#endif
    // gate prologue + modulus switching (lwe-bootstrapping-functions-fft.cu:1851-1858)
    for (int i = tid; i < kn; i += kV6Threads) {
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
    if (tid < 2) sh.sync[tid] = 0;
    for (int e = threadIdx.x; e < kT8Words; e += C * kV6Threads) shtw[e] = g.tw[t8_src(e)];
    const Tw4 tA = load_tw_sgpr(g.tw);
    __syncthreads();
    // ACC = (0, X^{2N - barb} (mu, ..., mu)) (:1427-1431)
    uint32_t acc[16];
    {
        const int e = (k2N - sh.barb) & (k2N - 1);
#pragma unroll
        for (int r = 0; r < 16; ++r)
            acc[r] = w == 0 ? 0u : (((L + 64 * r - e) & (k2N - 1)) < kN ? (uint32_t)mu : 0u - (uint32_t)mu);
    }
#ifdef TFHE_AMD_V6_STAMPS
    V6Stamps stamps;
    stamps.prev = __builtin_amdgcn_s_memtime();
#endif
    const int prio = g.prio;
    double mx = 0.0;                     // largest rounding distance of this lane (guard)
    uint32_t hlo = kQShiftHiLo, hhi = kQShiftHiLo;   // range of the rounding shifter's high word (guard)
    uint32_t bad = 0;                    // some coefficient's round(4c) != 0 mod 4 (distance >= 1/8)
    int a_next = sh.bara[0];
    int own = w;                         // this wave's LDS buffer (the waves swap every step)
    int seq = 0;                         // PS: partial sums handed over so far
    for (int i = 0; i < kn; ++i) {
        const int a = a_next;
        a_next = sh.bara[i + 1 < kn ? i + 1 : i];   // a step ahead: no LDS round trip at the loop head
        if (prio == 1) {
            if ((i & 127) == 0) set_prio_level(3 - (i >> 7));
        } else if (prio == 5) {   // rank on the CU (dispatch order) sets the phase
            if ((i & ((1 << g.prio_shift) - 1)) == 0)
                set_prio_level(2u * (unsigned)(blockIdx.x / g.cus) + ((unsigned)i >> g.prio_shift));
        }
        if (C == 1 && a == 0) continue;  // X^0 - 1 = 0: identity CMux (:705)
        cmux_v6<WAVES, RREG, RREG && C == 1, PS>(sh, shtw, g, tA, i, a, w, own, L, acc, mx, hlo, hhi, bad,
                                                 seq V6_STAMPS_ARG);
    }
    if (g.flags && live) {   // exactness guard: this wave's largest rounding distance (high word)
        if (bad || hlo < kQShiftHiLo || hhi >= kQShiftHiEnd) mx = 0.5;   // a distance >= 1/8, or |c| >= 2^49
        const uint32_t h = wave_max_hi(mx);
        if (L == 0) {
            g.flags[2 * slot + w] = h;
            atomicMax(g.stats + 1, h);
        }
    }
#ifdef TFHE_AMD_V6_STAMPS
    if (blockIdx.x == 0 && blockIdx.y == 0 && L == 0)
        for (int k = 0; k < 10; ++k) g_v6_stamps[w][k] += stamps.acc[k];
#endif
    // sample extraction at index 0 (lwe.cu:41-56): a_j = -acc_a[N - j] = E_a[2N - j]; the other
    // wave may still be in its last inverse in either buffer
    __syncthreads();
    if (!live) {
    } else if (w == 0) {
        uint32_t *E = reinterpret_cast<uint32_t *>(sh.X[0]);
        write_ext(E, acc, L);
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int j = L + 64 * r;
            ua[j] = (int32_t)E[(k2N - j) & (k2N - 1)];
        }
    } else if (L == 0) {
        *ub = (int32_t)acc[0];
    }
#ifdef TFHE_AMD_V6_STAMPS
    if (tid == 0 && wg < kWgSlots) {
        g_v6_wg[wg][1] = __builtin_amdgcn_s_memrealtime();
        g_v6_wg[wg][3] = __builtin_amdgcn_s_memtime();
    }
#endif
}

template <int WAVES, bool RREG>
__global__ __launch_bounds__(kV6Threads, WAVES) void k_blind_rotate_v6(V6Args g, int B, int base, BrInput in0,
                                                                BrInput in1, int32_t mu, int32_t *__restrict__ u_a,
                                                                int32_t *__restrict__ u_b) {
    __shared__ V6Shared sh;
    const int gct = base + blockIdx.x;
    const int half = gct >= B;
    const int idx = half ? gct - B : gct;
    const BrInput &in = half ? in1 : in0;
    RowTerms6 t;
    t.c = in.c; t.sa = in.sa; t.sb = in.sb; t.sc = 0;
    t.xa = in.x_a + (size_t)idx * kn; t.xb = in.x_b + idx;
    t.ya = in.sb ? in.y_a + (size_t)idx * kn : nullptr; t.yb = in.sb ? in.y_b + idx : nullptr;
    t.za = nullptr; t.zb = nullptr;
    br_v6_body<WAVES, RREG>(sh.ct[0], sh.tw, g, t, mu, u_a + (size_t)gct * kN, u_b + gct, (size_t)gct);
}

// two ciphertexts per workgroup (4 waves): the dispatcher spreads a 4-wave workgroup over the
// CU's 4 SIMDs, where two 2-wave workgroups sharing a CU land on 3 of them (2, 1, 1, 0 waves;
// scripts/wave_placement.hip), so at B <= 2 CUs this keeps one wave per SIMD
template <int WAVES, bool PS = false>
__global__ __launch_bounds__(2 * kV6Threads, WAVES) void k_blind_rotate_v6p(V6Args g, int B, int total, int base,
                                                                     BrInput in0, BrInput in1, int32_t mu,
                                                                     int32_t *__restrict__ u_a,
                                                                     int32_t *__restrict__ u_b) {
    __shared__ V6SharedC<2> sh;
    const int s = __builtin_amdgcn_readfirstlane(threadIdx.x >> 7);
    int gct = base + 2 * (int)blockIdx.x + s;
    const bool live = gct < total;
    if (!live) gct = total - 1;
    const int half = gct >= B;
    const int idx = half ? gct - B : gct;
    const BrInput &in = half ? in1 : in0;
    RowTerms6 t;
    t.c = in.c; t.sa = in.sa; t.sb = in.sb; t.sc = 0;
    t.xa = in.x_a + (size_t)idx * kn; t.xb = in.x_b + idx;
    t.ya = in.sb ? in.y_a + (size_t)idx * kn : nullptr; t.yb = in.sb ? in.y_b + idx : nullptr;
    t.za = nullptr; t.zb = nullptr;
    br_v6_body<WAVES, true, 2, PS>(sh.ct[s], sh.tw, g, t, mu, u_a + (size_t)gct * kN, u_b + gct, (size_t)gct, live);
}

template <int WAVES, bool RREG>
__global__ __launch_bounds__(kV6Threads, WAVES) void k_blind_rotate_v6_rows(V6Args g, int B, long base,
                                                                     const CircRow *__restrict__ rows,
                                                                     const int32_t *__restrict__ wa,
                                                                     const int32_t *__restrict__ wb, int32_t mu,
                                                                     int32_t *__restrict__ u_a,
                                                                     int32_t *__restrict__ u_b) {
    __shared__ V6Shared sh;
    const long flat = base + blockIdx.x;          // row-major (row, instance)
    const int r = (int)(flat / B), k = (int)(flat - (long)r * B);
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
    const size_t slot = (size_t)r * B + k;
    br_v6_body<WAVES, RREG>(sh.ct[0], sh.tw, g, t, mu, u_a + slot * kN, u_b + slot, slot);
}

template <bool RREG>
__global__ __launch_bounds__(kV6Threads, 2) void k_blind_rotate_v6_debug(V6Args g, int iters, int32_t *__restrict__ acc,
                                                                      const int32_t *__restrict__ bara) {
    __shared__ V6Shared sh;
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = tid & 63;
    int32_t *accg = acc + (size_t)blockIdx.x * 2 * kN + (size_t)w * kN;
    uint32_t ac[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) ac[r] = (uint32_t)accg[L + 64 * r];
    for (int i = tid; i < iters; i += kV6Threads) sh.ct[0].bara[i] = (short)(bara[(size_t)blockIdx.x * iters + i] & (k2N - 1));
    for (int e = tid; e < kT8Words; e += kV6Threads) sh.tw[e] = g.tw[t8_src(e)];
    const Tw4 tA = load_tw_sgpr(g.tw);
    __syncthreads();
    int own = w;
    for (int i = 0; i < iters; ++i) {
        const int a = sh.ct[0].bara[i];
        if (a == 0) continue;
#ifdef TFHE_AMD_V6_STAMPS
        V6Stamps stamps;
#endif
        double mx = 0.0;
        uint32_t hlo = kQShiftHiLo, hhi = kQShiftHiLo, bad = 0;
        // RREG: the throughput launches' form (the scalar-branch permutation, RSW), so that the
        // forced rotation edges of test_register_rotation_edges reach it
        int seq = 0;
        cmux_v6<2, RREG, RREG>(sh.ct[0], sh.tw, g, tA, i, a, w, own, L, ac, mx, hlo, hhi, bad, seq V6_STAMPS_ARG);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) accg[L + 64 * r] = (int32_t)ac[r];
}


// key conversion: one wave per (i, row, c) polynomial; z_n = b_n + i b_{n + 512} -> FFT / 512
__global__ __launch_bounds__(64) void k_bk_to_fft(const int32_t *__restrict__ bk_coef, double2 *__restrict__ bkf,
                                                  const double2 *__restrict__ tw) {
    __shared__ double2 X[kXSlots];
    const int poly = blockIdx.x;          // (i * 4 + row) * 2 + c, the coefficient layout's order
    const int L = threadIdx.x;
    const int32_t *src = bk_coef + (size_t)poly * kN;
    Cx x[1][8];
#pragma unroll
    for (int r = 0; r < 8; ++r) x[0][r] = Cx{(double)src[L + 64 * r], (double)src[L + 64 * r + 512]};
    fft_fwd_AB<1>(x, X, tw, load_tw_sgpr(tw), L);
    fft_fwd_C<1>(x, load_tw(tw, 1, L));
    double2 *dst = bkf + (size_t)poly * 512 + L;
#pragma unroll
    for (int r = 0; r < 8; ++r) st(dst + r * 64, Cx{x[0][r].re * (1.0 / 512), x[0][r].im * (1.0 / 512)});
}

}  // namespace

// Twiddles of the merged-twist transform (scripts/emu_v6.py twiddles_v6): angles in units of
// 2 pi / 8192; block b of stage s has modulus X^(2h) - C[s][b]; even blocks take the principal
// square root, odd blocks i x their even sibling (only even-block twiddles are stored).
void build_v6_twiddles(double2 *tw) {
    constexpr int M = 8192;
    std::vector<int> C{2048};
    std::vector<std::vector<int>> W;
    for (int s = 0; s < 9; ++s) {
        std::vector<int> ws(C.size());
        for (size_t b = 0; b < C.size(); ++b) ws[b] = (b % 2 == 0) ? C[b] / 2 : (ws[b - 1] + 2048) % M;
        std::vector<int> nc;
        for (int x : ws) { nc.push_back(x); nc.push_back((x + M / 2) % M); }
        W.push_back(ws);
        C = nc;
    }
    auto cis = [&](int e) {
        const long double th = 2.0L * 3.14159265358979323846264338327950288L * (long double)e / (long double)M;
        return make_double2((double)cosl(th), (double)sinl(th));
    };
    tw[0] = cis(W[0][0]);
    tw[1] = cis(W[1][0]);
    tw[2] = cis(W[2][0]);
    tw[3] = cis(W[2][2]);
    auto cexp = [](long double num, long double den) {   // e^{-2 pi i num / den}
        const long double th = -2.0L * 3.14159265358979323846264338327950288L * num / den;
        return make_double2((double)cosl(th), (double)sinl(th));
    };
    for (int L = 0; L < 64; ++L) {
        const int l7 = L & 7;
        tw[kTwInv + 0 * 64 + L] = cexp(l7, 16);
        tw[kTwInv + 1 * 64 + L] = cexp(l7, 32);
        tw[kTwInv + 2 * 64 + L] = cexp(l7, 64);
        tw[kTwInv + 3 * 64 + L] = cexp(8 * l7 + 64, 512);          // c e^{-i pi / 4}
        tw[kTwInv + 256 + 0 * 64 + L] = cexp(L, 128);
        tw[kTwInv + 256 + 1 * 64 + L] = cexp(L, 256);
        tw[kTwInv + 256 + 2 * 64 + L] = cexp(L, 512);
        tw[kTwInv + 256 + 3 * 64 + L] = cexp(L + 64, 512);
        for (int r = 0; r < 8; ++r) tw[kTwPost + r * 64 + L] = cexp(L + 64 * r, 2048);   // zeta^-n
        tw[kTwSig + L] = cexp(L, 2048);                             // zeta^-L
        tw[kTwInvAs + L] = cexp(17 * L, 2048);                      // e^{-2 pi i L / 128} zeta^-L
    }
    for (int L = 0; L < 64; ++L) {
        const int g = L >> 3;
        tw[4 + 0 * 64 + L] = cis(W[3][g]);
        tw[4 + 1 * 64 + L] = cis(W[4][2 * g]);
        tw[4 + 2 * 64 + L] = cis(W[5][4 * g]);
        tw[4 + 3 * 64 + L] = cis(W[5][4 * g + 2]);
        tw[4 + 256 + 0 * 64 + L] = cis(W[6][L]);
        tw[4 + 256 + 1 * 64 + L] = cis(W[7][2 * L]);
        tw[4 + 256 + 2 * 64 + L] = cis(W[8][4 * L]);
        tw[4 + 256 + 3 * 64 + L] = cis(W[8][4 * L + 2]);
    }
}

hipError_t launch_bk_to_fft(const int32_t *d_bk_coef, double2 *d_bkf, const double2 *d_tw, hipStream_t s) {
    hipLaunchKernelGGL(k_bk_to_fft, dim3(kn * kKpl * 2), dim3(64), 0, s, d_bk_coef, d_bkf, d_tw);
    return hipGetLastError();
}

// Launch geometry.  4 workgroups fit a CU (VGPRs and LDS); a launch of more than one round of
// workgroups is split into launches of one round each (4 x CUs ciphertexts), each balanced by
// the rank-phased rotation (policy 5): B = 4096 11.8-12.4 ms, against 13.4 with the hashed
// rotation and >= 13.5 for one launch with the by-step policy.
static int v6_cus(const DeviceKey &key) {
    static std::atomic<int> cus[64];   // per device; concurrent first calls store the same value
    const bool cached = key.device >= 0 && key.device < 64;
    int n = cached ? cus[key.device].load(std::memory_order_relaxed) : 0;
    if (!n) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, key.device) != hipSuccess || n <= 0) n = 256;
        if (cached) cus[key.device].store(n, std::memory_order_relaxed);
    }
    return n;
}
static long v6_chunk(const DeviceKey &key) { return 4L * v6_cus(key); }
// Two ciphertexts per workgroup (k_blind_rotate_v6p) for a launch of n ciphertexts when
// CUs < n <= 2 CUs: then at most one 4-wave workgroup per CU, one wave per SIMD, where 2-wave
// workgroups would pair up on some CUs over 3 SIMDs (B = 512: 2.36 -> 2.30 ms).  At n <= CUs
// one 2-wave workgroup per CU is faster (B = 256: 1.74 vs 2.29 ms: 2 waves on a CU run each step
// faster than 4 — LDS and the key path are shared per CU), and above 2 CUs the 2-wave
// workgroups fill every SIMD (B = 768: 2.62 vs 3.18 ms, 1024: 3.12 vs 3.26).
static bool v6_pair(const DeviceKey &key, long n) {
    const long cus = v6_cus(key);
    return n > cus && n <= 2 * cus;
}
// the register / ds_bpermute rotation (cmux_v6 RREG) for launches of more than one workgroup
// per CU; TFHE_AMD_V6_RREG=0/1 forces it off/on (experiments, tests)
// the paired kernel's waves meet per ciphertext through LDS counters instead of the workgroup
// barrier (cmux_v6 PS): B = 512 2.004 vs 2.277 ms, B = 384 1.995 vs 2.274 (profiles/r04j_pairsync_ab.txt);
// TFHE_AMD_V6P_PAIRSYNC=0 restores the barrier
static bool v6p_pairsync() {
    static const char *env = getenv("TFHE_AMD_V6P_PAIRSYNC");
    return env ? atoi(env) != 0 : true;
}
// (the one-ciphertext kernel's two waves through the same LDS counters, where the barrier couples
// only the ciphertext's own two waves, measured no faster: B = 1 024 3.039 vs 3.010 ms, B = 1 / 64
// / 256 1.676 / 1.713 / 1.726 vs 1.642 / 1.693 / 1.695 ms — a barrier between two waves in step is
// cheaper than polling: profiles/r04k_v6_pairsync_ab.txt, r04w_v6_pairsync_small_ab.txt)
static bool v6_rreg(const DeviceKey &key, long n) {
    static const char *env = getenv("TFHE_AMD_V6_RREG");
    if (env) return atoi(env) != 0;
    return n > v6_cus(key);
}
// (the paired kernel, one wave per SIMD, has no SIMD partner to arbitrate against: no policy,
// B = 512 1.984-1.991 vs 2.003-2.005 ms with policy 5, profiles/r04r_prio_sweep.txt)
static int v6_prio_policy(const DeviceKey &key, long wgs, bool paired = false) {
    if (paired) return 0;
    return wgs > 4L * v6_cus(key) ? 1 : 5;
}

// policy 5's steps per priority level = 2^kV6PrioShift (variant builds: -DTFHE_AMD_V6_PRIO_SHIFT=n)
#ifndef TFHE_AMD_V6_PRIO_SHIFT
#define TFHE_AMD_V6_PRIO_SHIFT 3
#endif
constexpr int kV6PrioShift = TFHE_AMD_V6_PRIO_SHIFT;
static V6Args v6_args(const DeviceKey &key, long wgs, const Guard *guard = nullptr, bool paired = false) {
    V6Args g;
    g.bk = key.bk_fft;
    g.flags = guard ? guard->flags : nullptr;
    g.stats = guard ? guard->stats : nullptr;
    g.tw = key.tw6;
    g.prio = wgs > 0 ? v6_prio_policy(key, wgs, paired) : 0;
    g.prio_shift = kV6PrioShift;
    g.cus = v6_cus(key);
    return g;
}

hipError_t launch_blind_rotate_v6(const DeviceKey &key, int B, int halves, const BrInput *in, int32_t mu,
                                  int32_t *u_a, int32_t *u_b, hipStream_t s, const Guard *guard) {
    if (B <= 0) return hipSuccess;
    if (!key.bk_fft) return hipErrorInvalidValue;
    const BrInput in1 = halves > 1 ? in[1] : in[0];
    const long total = (long)B * halves, chunk = v6_chunk(key);
    for (long base = 0; base < total; base += chunk) {
        const long n = total - base < chunk ? total - base : chunk;
        if (v6_pair(key, n)) {
            const long wgs = (n + 1) / 2;
            // the pair sync's bounded poll hands a ciphertext whose partner never arrives to the
            // guard (bad flag -> exact recomputation): only with guard flags to hand it to
            if (v6p_pairsync() && guard && guard->flags) {
                trace_kernel("k_blind_rotate_v6p(paired+reg-rotation+pair-sync)");
                hipLaunchKernelGGL((k_blind_rotate_v6p<kV6Waves, true>), dim3((unsigned)wgs), dim3(2 * kV6Threads), 0, s,
                                   v6_args(key, wgs, guard, true), B, (int)total, (int)base, in[0], in1, mu, u_a, u_b);
            } else {
                trace_kernel("k_blind_rotate_v6p(paired+reg-rotation)");
                hipLaunchKernelGGL(k_blind_rotate_v6p<kV6Waves>, dim3((unsigned)wgs), dim3(2 * kV6Threads), 0, s,
                                   v6_args(key, wgs, guard, true), B, (int)total, (int)base, in[0], in1, mu, u_a, u_b);
            }
        } else {
            trace_kernel(v6_rreg(key, n) ? "k_blind_rotate_v6(reg-rotation)" : "k_blind_rotate_v6(lds-rotation)");
            if (v6_rreg(key, n))
                hipLaunchKernelGGL((k_blind_rotate_v6<kV6Waves, true>), dim3((unsigned)n), dim3(kV6Threads), 0, s,
                                   v6_args(key, n, guard), B, (int)base, in[0], in1, mu, u_a, u_b);
            else
                hipLaunchKernelGGL((k_blind_rotate_v6<kV6Waves, false>), dim3((unsigned)n), dim3(kV6Threads), 0, s,
                                   v6_args(key, n, guard), B, (int)base, in[0], in1, mu, u_a, u_b);
        }
    }
    return hipGetLastError();
}

hipError_t launch_blind_rotate_v6_rows(const DeviceKey &key, int B, int nrows, const CircRow *rows, const int32_t *wa,
                                       const int32_t *wb, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t s,
                                       const Guard *guard) {
    if (B <= 0 || nrows <= 0) return hipSuccess;
    if (!key.bk_fft) return hipErrorInvalidValue;
    const long total = (long)B * nrows, chunk = v6_chunk(key);
    for (long base = 0; base < total; base += chunk) {
        const long n = total - base < chunk ? total - base : chunk;
        if (n > 0x7fffffffL) return hipErrorInvalidValue;
        trace_kernel(v6_rreg(key, n) ? "k_blind_rotate_v6_rows(reg-rotation)" : "k_blind_rotate_v6_rows(lds-rotation)");
        if (v6_rreg(key, n))
            hipLaunchKernelGGL((k_blind_rotate_v6_rows<kV6Waves, true>), dim3((unsigned)n), dim3(kV6Threads), 0, s,
                               v6_args(key, n, guard), B, base, rows, wa, wb, mu, u_a, u_b);
        else
            hipLaunchKernelGGL((k_blind_rotate_v6_rows<kV6Waves, false>), dim3((unsigned)n), dim3(kV6Threads), 0, s,
                               v6_args(key, n, guard), B, base, rows, wa, wb, mu, u_a, u_b);
    }
    return hipGetLastError();
}

hipError_t launch_blind_rotate_v6_debug(const DeviceKey &key, int B, int iters, int32_t *acc, const int32_t *bara,
                                        hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (iters < 0 || iters > kn || !key.bk_fft) return hipErrorInvalidValue;
    trace_kernel(v6_rreg(key, B) ? "k_blind_rotate_v6_debug(reg-rotation)" : "k_blind_rotate_v6_debug(lds-rotation)");
    if (v6_rreg(key, B))
        hipLaunchKernelGGL(k_blind_rotate_v6_debug<true>, dim3(B), dim3(kV6Threads), 0, s, v6_args(key, 0), iters, acc,
                           bara);
    else
        hipLaunchKernelGGL(k_blind_rotate_v6_debug<false>, dim3(B), dim3(kV6Threads), 0, s, v6_args(key, 0), iters,
                           acc, bara);
    return hipGetLastError();
}

}  // namespace tfhe_amd

#ifdef TFHE_AMD_V6_STAMPS
extern "C" int tfhe_amd_debug_v6_stamps(unsigned long long *out, int reset) {
    unsigned long long h[24];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(tfhe_amd::g_v6_stamps), sizeof h) != hipSuccess) return -2;
    for (int i = 0; i < 24; i++) out[i] = h[i];
    if (reset) {
        unsigned long long z[24] = {0};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(tfhe_amd::g_v6_stamps), z, sizeof z);
    }
    return 0;
}
extern "C" int tfhe_amd_debug_v6_wgtime(unsigned long long *out, int n) {
    if (n > tfhe_amd::kWgSlots) n = tfhe_amd::kWgSlots;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(tfhe_amd::g_v6_wg), (size_t)n * 6 * sizeof(unsigned long long)) ==
                   hipSuccess
               ? 0
               : -2;
}
#endif
