// blind_rotate_v4.hip — v4 blind rotation: v2's register-resident layout with fewer VALU
// instructions per CMux step (the v2 kernel is VALU-issue bound: its time tracks its
// instruction count).
//
// Same contract as v2 (tfhe_blindRotate_FFT + extraction, lwe-bootstrapping-functions-fft.cu
// :676-737, 1408-1456, 1834-1870; tGswFFTExternMulToTLwe tgsw-fft-operations.cu:124-264).
// Changes against v2, all exact (scripts/emu_v4.py checks the index math and the bounds):
//  * inverse transform = Cooley-Tukey DIT on the bit-reversed slots + a psi^-n post-twist
//    (5 VALU per butterfly, no reductions: < 23.75q) instead of Harvey Gentleman-Sande (8);
//  * the MAC's REDC result stays lazy (< 3.75q), the inverse output stays lazy ([0, 2q)) and
//    the CRT lift takes both residues lazily;
//  * the accumulator is kept as a periodic negacyclic extension E[k] = +-acc[k mod N]
//    (k < 3N, sign - when k mod 2N >= N): X^a * ACC at coefficient j is E[(j - a) mod 2N + ...]
//    read with immediate offsets, so the rotation costs no address or sign arithmetic.
#include "engine.h"
#include "modarith.h"
#include "ntt_wave.h"

namespace tfhe_amd {

namespace {

constexpr int kV4Threads = 128;
constexpr int kExt = 3 * kN;

struct V4Shared {
    uint32_t E[2][kExt];               // periodic negacyclic accumulator (a, b), 24 KB
    uint32_t scratch[2][kPadRow];      // one per wave (prime)
    int bara[512];
    int barb;
};

struct V4Args {
    const uint32_t *bk;   // [kn][2][2 c][4 p][4 v][64 L][4 e]   (v2 layout)
    const uint2 *tu_f;    // [2][16] uniform forward twiddles (negated)
    const uint2 *ts_f;    // [2][27][64] forward streams (negated)
    const uint2 *tu_i;    // [2][16] inverse-CT uniform twiddles (negated)
    const uint2 *ts_i;    // [2][27][64] inverse-CT streams (negated)
    const uint2 *tpost;   // [2][16][64] psi^-(L + 64 r), positive
    uint32_t qinv_neg0, qinv_neg1, crt_h, crt_hp;
};

__device__ __forceinline__ void e_store(uint32_t *E, int j, uint32_t v) {
    E[j] = v;
    E[j + kN] = 0u - v;
    E[j + 2 * kN] = v;
}

// centred CRT lift of lazy residues x0 in [0, 2 q0), x1 in [0, 2 q1), reduced mod 2^32.
// The exact external-product coefficient c has |c| < 2^52 << q0 q1 / 2, so the lift
// x0 + q0 tc with tc = (x1 - x0) q0^-1 mod q1 taken in (-q1/2, q1/2] equals c.
__device__ __forceinline__ uint32_t crt_lazy(uint32_t x0, uint32_t x1, uint32_t h, uint32_t hp) {
    const uint32_t d = x1 + 3u * kQ1 - x0;                      // (q1, 5 q1)
    const uint32_t t0 = shoup_lazy(d, h, hp, 0u - kQ1);         // [0, 2 q1)
    const uint32_t t = umin32(t0, t0 - kQ1);                    // [0, q1)
    const uint32_t tc = t > (kQ1 - 1) / 2 ? t - kQ1 : t;
    return x0 + kQ0 * tc;
}

template <int S>
__device__ __forceinline__ void crt4_give(V4Shared &sh, const uint32_t (&O)[2][16], int L) {
    uint32_t *mine = sh.scratch[S];
    constexpr int give = 8 * (1 - S);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) mine[(c * 8 + rr) * 64 + L] = O[c][give + rr];
}
// XP (external product only, tGswFFTExternMulToTLwe): the result replaces the accumulator
template <int S, bool XP = false>
__device__ __forceinline__ void crt4_take(V4Shared &sh, const uint32_t (&O)[2][16], int L, const V4Args &g) {
    const uint32_t *other = sh.scratch[1 - S];
    constexpr int keep = 8 * S;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) {
            const uint32_t xo = other[(c * 8 + rr) * 64 + L];
            const uint32_t xm = O[c][keep + rr];
            const uint32_t x0 = S == 0 ? xm : xo, x1 = S == 0 ? xo : xm;
            const int j = L + 64 * (keep + rr);
            e_store(sh.E[c], j, (XP ? 0u : sh.E[c][j]) + crt_lazy(x0, x1, g.crt_h, g.crt_hp));
        }
}

// one CMux step for key index i and rotation a (1..2N-1); called by both waves.  XP: the
// external product alone, ACC <- BK_i (x) ACC (tgsw-fft-operations.cu:124-264; a unused)
template <bool XP = false>
__device__ __forceinline__ void cmux_v4(V4Shared &sh, const V4Args &g, int i, int a, int s, int L) {
    const uint32_t q = s ? kQ1 : kQ0;
    uint32_t *sc = sh.scratch[s];
    // (X^a - 1) ACC + gadget decomposition (tgsw-functions.cu:300-413), layout A; digits
    // lifted to [q - 512, q + 511]
    uint32_t D[4][16];
    const int base = (L - a) & (k2N - 1);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t t = (XP ? 0u : sh.E[c][base + 64 * r] - sh.E[c][L + 64 * r]) +
                               (XP ? sh.E[c][L + 64 * r] : 0u) + kDecompOffset;
            D[2 * c][r] = ((t >> 22) & 1023u) + (q - 512u);
            D[2 * c + 1][r] = ((t >> 12) & 1023u) + (q - 512u);
        }
    const uint2 *tsf = g.ts_f + s * 27 * 64 + L, *tsi = g.ts_i + s * 27 * 64 + L, *tpb = g.tpost + s * 16 * 64 + L;
    ntt_fwd<4>(D, sc, g.tu_f + 16 * s, tsf, L, q);
    // pointwise MAC with BK_i (layout C: reg r = 4 v + e <-> slot 16 L + r), REDC lazy
    const uint4 *bk4 = reinterpret_cast<const uint4 *>(g.bk + ((size_t)(i * 2 + s) * 8) * kN) + L;
    const uint32_t qinv = s ? g.qinv_neg1 : g.qinv_neg0;
    uint32_t O[2][16];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            uint4 b[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) b[p] = bk4[(c * 4 + p) * 256 + v * 64];
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
                O[c][r] = (uint32_t)((x + (uint64_t)m * q) >> 32);               // < 3.75 q
            }
        }
    }
    ntt_inv_ct<2>(O, sc, g.tu_i + 16 * s, tsi, L, q);   // < 31.75 q, layout A
    {   // post-twist psi^-n (n = L + 64 r) -> [0, 2q)
        const uint2 *tp = tpb;
        const uint32_t negq = 0u - q;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint2 w = tp[r * 64];
#pragma unroll
            for (int c = 0; c < 2; ++c) O[c][r] = shoup_lazy(O[c][r], w.x, w.y, negq);
        }
    }
    if (s == 0) crt4_give<0>(sh, O, L);
    else crt4_give<1>(sh, O, L);
    __syncthreads();
    if (s == 0) crt4_take<0, XP>(sh, O, L, g);
    else crt4_take<1, XP>(sh, O, L, g);
    __syncthreads();
}

// The linear combination x = (0, c) + sa X + sb Y + sc Z that feeds one blind rotation
// (gate prologues boot-gates.cu:98-448; a circuit row adds a third input for MAJ / XOR3).
struct RowTerms {
    int32_t c, sa, sb, sc;
    const int32_t *xa, *xb, *ya, *yb, *za, *zb;   // a rows (kn) and b words; y/z may be null
};

// prologue + modswitch + 500 CMux steps + extraction of one ciphertext into (ua, *ub)
__device__ __forceinline__ void br_v4_body(V4Shared &sh, const V4Args &g, const RowTerms &t, int32_t mu,
                                           int32_t *__restrict__ ua, int32_t *__restrict__ ub) {
    const int tid = threadIdx.x;
    const int s = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = tid & 63;
    // gate prologue + modulus switching (lwe-bootstrapping-functions-fft.cu:1851-1858)
    for (int i = tid; i < kn; i += kV4Threads) {
        uint32_t x = t.xa ? (uint32_t)t.sa * (uint32_t)t.xa[i] : 0u;
        if (t.ya) x += (uint32_t)t.sb * (uint32_t)t.ya[i];
        if (t.za) x += (uint32_t)t.sc * (uint32_t)t.za[i];
        sh.bara[i] = modswitch_2N(x);
    }
    if (tid == 0) {
        uint32_t xb = (uint32_t)t.c + (t.xb ? (uint32_t)t.sa * (uint32_t)t.xb[0] : 0u);
        if (t.yb) xb += (uint32_t)t.sb * (uint32_t)t.yb[0];
        if (t.zb) xb += (uint32_t)t.sc * (uint32_t)t.zb[0];
        sh.barb = modswitch_2N(xb);
    }
    __syncthreads();
    {   // ACC = (0, X^{2N - barb} (mu, ..., mu)) (:1427-1431), as its periodic extension
        const int e = (k2N - sh.barb) & (k2N - 1);
        for (int k = tid; k < kExt; k += kV4Threads) {
            sh.E[0][k] = 0;
            sh.E[1][k] = ((k - e) & (k2N - 1)) < kN ? (uint32_t)mu : 0u - (uint32_t)mu;
        }
    }
    __syncthreads();
    for (int i = 0; i < kn; ++i) {
        const int a = sh.bara[i];
        if (a == 0) continue;            // X^0 - 1 = 0: identity CMux (:705)
        cmux_v4(sh, g, i, a, s, L);
    }
    // sample extraction at index 0 (lwe.cu:41-56): a_j = -acc_a[N - j] = E_a[2N - j]
    for (int j = tid; j < kN; j += kV4Threads) ua[j] = (int32_t)sh.E[0][(k2N - j) & (k2N - 1)];
    if (tid == 0) *ub = (int32_t)sh.E[1][0];
}

// Guard mode (engine.h Guard): the fp64 kernel ran first and flagged each ciphertext with its
// largest rounding distance; a ciphertext under the threshold keeps its result (the workgroup
// exits before touching anything), one at or above it is recomputed here exactly.
struct V4Guard {
    const uint32_t *flags;   // null: not in guard mode
    uint32_t hi;             // threshold (high word of the distance)
    uint32_t *stats;         // [0]: recomputed ciphertexts
};
__device__ __forceinline__ bool guard_skip(const V4Guard &gd, size_t slot) {
    if (!gd.flags) return false;
    const uint32_t f0 = gd.flags[2 * slot], f1 = gd.flags[2 * slot + 1];
    if ((f0 > f1 ? f0 : f1) < gd.hi) return true;   // uniform over the workgroup
    if (threadIdx.x == 0) atomicAdd(gd.stats, 1u);
    return false;
}

// gate batch: ciphertext gct of half h = gct / B reads in_h at index gct mod B.  Grid-stride
// over the total ciphertexts: one per workgroup normally; in guard mode a small grid scans the
// flags (almost always all clear) instead of dispatching one workgroup per ciphertext.
// MINW: waves per SIMD the register budget is cut for — 2 for the exact throughput kernel
// (tfhe_amd_select_kernel(4): 256 VGPRs, 27 spilled), 1 for the guard launch (284 VGPRs, no scratch: a
// kernel with a private segment costs ~12 us more per dispatch even when every workgroup exits
// at once)
template <int MINW>
__global__ __launch_bounds__(kV4Threads, MINW) void k_blind_rotate_v4(V4Args g, int B, int total, BrInput in0,
                                                                BrInput in1, int32_t mu,
                                                                int32_t *__restrict__ u_a,
                                                                int32_t *__restrict__ u_b, V4Guard gd) {
    __shared__ V4Shared sh;
    bool used = false;
    for (int gct = blockIdx.x; gct < total; gct += gridDim.x) {
        if (guard_skip(gd, (size_t)gct)) continue;
        if (used) __syncthreads();   // the previous ciphertext's extraction has read the LDS
        used = true;
        const int half = gct >= B;
        const int idx = half ? gct - B : gct;
        const BrInput &in = half ? in1 : in0;
        RowTerms t;
        t.c = in.c; t.sa = in.sa; t.sb = in.sb; t.sc = 0;
        t.xa = in.x_a + (size_t)idx * kn; t.xb = in.x_b + idx;
        t.ya = in.sb ? in.y_a + (size_t)idx * kn : nullptr; t.yb = in.sb ? in.y_b + idx : nullptr;
        t.za = nullptr; t.zb = nullptr;
        br_v4_body(sh, g, t, mu, u_a + (size_t)gct * kN, u_b + gct);
    }
}

// circuit level: flat slot r B + k (row r, instance k < B), grid-stride as the gate kernel;
// wires are [W][B] ciphertexts, the extracted sample of (r, k) goes to u slot r B + k
template <int MINW>
__global__ __launch_bounds__(kV4Threads, MINW) void k_blind_rotate_v4_rows(V4Args g, int B, long total,
                                                                     const CircRow *__restrict__ rows,
                                                                     const int32_t *__restrict__ wa,
                                                                     const int32_t *__restrict__ wb, int32_t mu,
                                                                     int32_t *__restrict__ u_a,
                                                                     int32_t *__restrict__ u_b, V4Guard gd) {
    __shared__ V4Shared sh;
    bool used = false;
    for (long slot = blockIdx.x; slot < total; slot += gridDim.x) {
        if (guard_skip(gd, (size_t)slot)) continue;
        if (used) __syncthreads();
        used = true;
        const int r = (int)(slot / B), k = (int)(slot - (long)r * B);
        const CircRow row = rows[r];
        auto wire = [&](int w, const int32_t *&pa, const int32_t *&pb) {
            if (w < 0) { pa = nullptr; pb = nullptr; return; }
            const size_t ws = (size_t)w * B + k;
            pa = wa + ws * kn;
            pb = wb + ws;
        };
        RowTerms t;
        t.c = row.c; t.sa = row.sa; t.sb = row.sb; t.sc = row.sc;
        wire(row.x, t.xa, t.xb);
        wire(row.y, t.ya, t.yb);
        wire(row.z, t.za, t.zb);
        br_v4_body(sh, g, t, mu, u_a + (size_t)slot * kN, u_b + slot);
    }
}

__global__ __launch_bounds__(kV4Threads, 2) void k_blind_rotate_v4_debug(V4Args g, int iters, int32_t *__restrict__ acc,
                                                                      const int32_t *__restrict__ bara) {
    __shared__ V4Shared sh;
    const int tid = threadIdx.x;
    const int s = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = tid & 63;
    int32_t *accg = acc + (size_t)blockIdx.x * 2 * kN;
    for (int j = tid; j < 2 * kN; j += kV4Threads) e_store(sh.E[j >> kLogN], j & (kN - 1), (uint32_t)accg[j]);
    for (int i = tid; i < iters; i += kV4Threads) sh.bara[i] = bara[(size_t)blockIdx.x * iters + i] & (k2N - 1);
    __syncthreads();
    for (int i = 0; i < iters; ++i) {
        const int a = sh.bara[i];
        if (a == 0) continue;
        cmux_v4(sh, g, i, a, s, L);
    }
    for (int j = tid; j < 2 * kN; j += kV4Threads) accg[j] = (int32_t)sh.E[j >> kLogN][j & (kN - 1)];
}

// tGswFFTExternMulToTLwe batch: accumulator b (acc [B][2][kN]) <- BK_{key_index[b]} (x) acc, exact
__global__ __launch_bounds__(kV4Threads, 2) void k_external_product_v4(V4Args g, const int32_t *__restrict__ key_index,
                                                                        int32_t *__restrict__ acc) {
    __shared__ V4Shared sh;
    const int tid = threadIdx.x;
    const int s = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = tid & 63;
    int32_t *accg = acc + (size_t)blockIdx.x * 2 * kN;
    // the index comes from device memory unchecked by the host: outside [0, kn) the accumulator is
    // left as it is (whole workgroup, uniform) rather than reading past the key
    const int i = key_index[blockIdx.x];
    if (i < 0 || i >= kn) return;
    for (int j = tid; j < 2 * kN; j += kV4Threads) e_store(sh.E[j >> kLogN], j & (kN - 1), (uint32_t)accg[j]);
    __syncthreads();
    cmux_v4<true>(sh, g, i, 0, s, L);
    for (int j = tid; j < 2 * kN; j += kV4Threads) accg[j] = (int32_t)sh.E[j >> kLogN][j & (kN - 1)];
}

unsigned brv10(unsigned x) {
    unsigned r = 0;
    for (int i = 0; i < kLogN; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

}  // namespace

// Inverse-CT and post-twist tables of the v4 kernel, host side, consumption order.
// psi^-m for m < N is ipsi[brv(m)] (ntt_tables.h).
void build_v4_twiddles(const NttTables &t, uint2 *tu_i, uint2 *ts_i, uint2 *tpost) {
    for (int s = 0; s < 2; ++s) {
        const uint32_t q = kQ[s];
        auto ipow = [&](unsigned m) { return t.ipsi[s][brv10(m)]; };
        auto shp = [&](uint32_t w) { return (uint32_t)(((uint64_t)w << 32) / q); };
        auto neg = [&](uint32_t w) { return make_uint2(0u - w, shp(w)); };
        tu_i[s * 16 + 15] = make_uint2(0, 0);
        for (int S = 0; S <= 3; ++S)
            for (int p = 0; p < (1 << S); ++p) tu_i[s * 16 + (1 << S) - 1 + p] = neg(ipow((unsigned)p << (10 - S)));
        int slot = 0;
        for (int S = 4; S <= 9; ++S) {
            const int cnt = S <= 5 ? 1 << (S - 2) : 1 << (S - 6);
            for (int g = 0; g < cnt; ++g, ++slot)
                for (int L = 0; L < 64; ++L) {
                    const unsigned p = S <= 5 ? (unsigned)((L & 3) | (g << 2)) : (unsigned)(L + 64 * g);
                    ts_i[(s * 27 + slot) * 64 + L] = neg(ipow(p << (10 - S)));
                }
        }
        for (int r = 0; r < 16; ++r)
            for (int L = 0; L < 64; ++L) {
                const uint32_t w = ipow((unsigned)(L + 64 * r));
                tpost[(s * 16 + r) * 64 + L] = make_uint2(w, shp(w));
            }
    }
}

static V4Args v4_args(const DeviceKey &key) {
    V4Args g;
    g.bk = key.bk_v2;
    g.tu_f = key.tw2;
    g.ts_f = key.tw2 + 64;
    g.tu_i = key.tw4;
    g.ts_i = key.tw4 + 32;
    g.tpost = key.tw4 + 32 + 2 * 27 * 64;
    g.qinv_neg0 = key.qinv_neg[0];
    g.qinv_neg1 = key.qinv_neg[1];
    g.crt_h = key.crt_h;
    g.crt_hp = key.crt_hp;
    return g;
}

constexpr int kGuardGrid = 256;
static V4Guard v4_guard(const Guard *guard) {
    V4Guard gd{nullptr, 0u, nullptr};
    if (guard && guard->flags) gd = V4Guard{guard->flags, guard_threshold_hi(), guard->stats};
    return gd;
}

hipError_t launch_blind_rotate_v4(const DeviceKey &key, int B, int halves, const BrInput *in, int32_t mu,
                                  int32_t *u_a, int32_t *u_b, hipStream_t s, const Guard *guard) {
    if (B <= 0) return hipSuccess;
    if (!key.bk_v2) return hipErrorInvalidValue;
    const BrInput in1 = halves > 1 ? in[1] : in[0];
    const V4Guard gd = v4_guard(guard);
    const int total = B * halves;
    // guard mode: 256 workgroups scan the flags (B = 1024: 15 -> ~4 us per launch)
    const int grid = gd.flags && total > kGuardGrid ? kGuardGrid : total;
    trace_kernel(gd.flags ? "k_blind_rotate_v4(guard)" : "k_blind_rotate_v4");
    if (gd.flags)
        hipLaunchKernelGGL(k_blind_rotate_v4<1>, dim3(grid), dim3(kV4Threads), 0, s, v4_args(key), B, total, in[0],
                           in1, mu, u_a, u_b, gd);
    else
        hipLaunchKernelGGL(k_blind_rotate_v4<2>, dim3(grid), dim3(kV4Threads), 0, s, v4_args(key), B, total, in[0],
                           in1, mu, u_a, u_b, gd);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_v4_rows(const DeviceKey &key, int B, int nrows, const CircRow *rows, const int32_t *wa,
                                       const int32_t *wb, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t s,
                                       const Guard *guard) {
    if (B <= 0 || nrows <= 0) return hipSuccess;
    if (!key.bk_v2) return hipErrorInvalidValue;
    const V4Guard gd = v4_guard(guard);
    const long total = (long)B * nrows;
    const long grid = gd.flags && total > kGuardGrid ? kGuardGrid : total < 0x7fffffffL ? total : 0x7fffffffL;
    trace_kernel(gd.flags ? "k_blind_rotate_v4_rows(guard)" : "k_blind_rotate_v4_rows");
    if (gd.flags)
        hipLaunchKernelGGL(k_blind_rotate_v4_rows<1>, dim3((unsigned)grid), dim3(kV4Threads), 0, s, v4_args(key), B,
                           total, rows, wa, wb, mu, u_a, u_b, gd);
    else
        hipLaunchKernelGGL(k_blind_rotate_v4_rows<2>, dim3((unsigned)grid), dim3(kV4Threads), 0, s, v4_args(key), B,
                           total, rows, wa, wb, mu, u_a, u_b, gd);
    return hipGetLastError();
}

hipError_t launch_external_product_v4(const DeviceKey &key, int B, const int32_t *key_index, int32_t *acc,
                                      hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (!key.bk_v2) return hipErrorInvalidValue;
    trace_kernel("k_external_product_v4");
    hipLaunchKernelGGL(k_external_product_v4, dim3(B), dim3(kV4Threads), 0, s, v4_args(key), key_index, acc);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_v4_debug(const DeviceKey &key, int B, int iters, int32_t *acc, const int32_t *bara,
                                        hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (iters < 0 || iters > kn) return hipErrorInvalidValue;
    trace_kernel("k_blind_rotate_v4_debug");
    hipLaunchKernelGGL(k_blind_rotate_v4_debug, dim3(B), dim3(kV4Threads), 0, s, v4_args(key), iters, acc, bara);
    return hipGetLastError();
}

}  // namespace tfhe_amd
