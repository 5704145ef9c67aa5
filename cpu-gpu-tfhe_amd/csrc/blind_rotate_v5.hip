// blind_rotate_v5.hip — latency-oriented blind rotation for small batches.
//
// v4 gives each ciphertext 2 waves (one per prime), so a CMux step costs a wave 4 forward
// NTTs + 2 inverse NTTs in sequence; that is the right shape when thousands of ciphertexts
// fill the chip, but a lone ciphertext (a circuit level of a single addition, B = 1 in the
// BASELINE metric) then waits ~9 us per step on two busy waves of one CU.  v5 spreads one
// ciphertext over 8 waves (512 threads, one CU):
//   wave w = 4 s + p   (s = prime, p = digit polynomial 2c + level)
//   1. every wave decomposes ITS digit polynomial and runs ONE forward NTT;
//   2. the NTT-domain digits meet in LDS (layout C, padded as in ntt_wave.h);
//   3. waves p = c < 2 form the MAC for output polynomial c of prime s (16 slots per lane,
//      BK_i 16-B loads issued one step ahead), run ONE inverse NTT and the post-twist;
//   4. waves (0, c) and (1, c) meet in the CRT exchange and update E (periodic accumulator).
// The critical path of a step is one forward + one inverse NTT instead of four + two.
// Arithmetic, layouts and tables are v4's (scripts/emu_v4.py), so results are identical.
#include "engine.h"
#include "modarith.h"
#include "ntt_wave.h"

namespace tfhe_amd {

namespace {

constexpr int kV5Threads = 512;

#ifdef TFHE_AMD_V5_STAMPS
// timing diagnostics: cumulative shader-clock cycles per phase for waves 0 (MAC) and 2 (idle)
// of workgroup 0; read with tfhe_amd_debug_v5_stamps
__device__ unsigned long long g_v5_stamps[2][12];
#define V5_STAMP(k)                                                                         \
    do {                                                                                     \
        if (blockIdx.x == 0 && blockIdx.y == 0 && (tid & 63) == 0 && (w == 0 || w == 2)) { \
            const unsigned long long now = __builtin_amdgcn_s_memtime();                     \
            g_v5_stamps[w >> 1][k] += now - t_prev;                                          \
            t_prev = now;                                                                    \
        }                                                                                    \
    } while (0)
#else
#define V5_STAMP(k) do {} while (0)
#endif
constexpr int kExt5 = 3 * kN;

struct V5Shared {
    uint32_t E[2][kExt5];              // periodic negacyclic accumulator (a, b), 24 KB
    uint32_t scratch[8][kPadRow];      // one per wave: NTT transposes, NTT-domain digit poly
                                       // (layout C padded), CRT exchange
    uint2 tsf[2][27][64];              // lane-stream twiddles, LDS-resident (latency: no L2
    uint2 tsi[2][27][64];              // round trip per NTT stage group), 72 KB in all
    uint2 tpost[2][16][64];
    int bara[512];
    int barb;
};

struct V5Args {
    const uint32_t *bk;   // v2 layout [kn][2][2 c][4 p][4 v][64 L][4 e]
    const uint2 *tu_f, *ts_f, *tu_i, *ts_i, *tpost;
    uint32_t qinv_neg0, qinv_neg1, crt_h, crt_hp;
};

__device__ __forceinline__ void e5_store(uint32_t *E, int j, uint32_t v) {
    E[j] = v;
    E[j + kN] = 0u - v;
    E[j + 2 * kN] = v;
}

__device__ __forceinline__ uint32_t crt5(uint32_t x0, uint32_t x1, uint32_t h, uint32_t hp) {
    const uint32_t d = x1 + 3u * kQ1 - x0;
    const uint32_t t0 = shoup_lazy(d, h, hp, 0u - kQ1);
    const uint32_t t = umin32(t0, t0 - kQ1);
    const uint32_t tc = t > (kQ1 - 1) / 2 ? t - kQ1 : t;
    return x0 + kQ0 * tc;
}

// BK_i slice of wave (s, c): 4 rows p x 4 v, one uint4 each (slot 16 L + 4 v + e)
__device__ __forceinline__ void load_bk(const V5Args &g, int i, int s, int c, int L, uint4 (&b)[4][4]) {
    const uint4 *bk4 = reinterpret_cast<const uint4 *>(g.bk + ((size_t)(i * 2 + s) * 8) * kN) + L;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int v = 0; v < 4; ++v) b[p][v] = bk4[(c * 4 + p) * 256 + v * 64];
}

// Workgroup barrier for LDS traffic only.  __syncthreads() is a workgroup-scope release /
// acquire fence around s_barrier, which also waits for every outstanding GLOBAL load
// (vmcnt(0)) — i.e. for the next step's BK_i prefetch, defeating it.  The step loop has no
// global stores, so an LDS-only wait + s_barrier is sufficient; the asm "memory" clobber
// keeps the compiler from moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int S>
__device__ __forceinline__ void crt5_give(uint32_t *sc, const uint32_t (&O)[16], int L) {
    constexpr int give = 8 * (1 - S);
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) sc[rr * 64 + L] = O[give + rr];
}
template <int S>
__device__ __forceinline__ void crt5_take(V5Shared &sh, const uint32_t *other, const uint32_t (&O)[16], int c, int L,
                                          const V5Args &g) {
    constexpr int keep = 8 * S;
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
        const uint32_t xo = other[rr * 64 + L];
        const uint32_t xm = O[keep + rr];
        const uint32_t x0 = S == 0 ? xm : xo, x1 = S == 0 ? xo : xm;
        const int jj = L + 64 * (keep + rr);
        e5_store(sh.E[c], jj, sh.E[c][jj] + crt5(x0, x1, g.crt_h, g.crt_hp));
    }
}

struct RowTerms5 {
    int32_t c, sa, sb, sc;
    const int32_t *xa, *xb, *ya, *yb, *za, *zb;
};

__device__ __forceinline__ void br_v5_body(V5Shared &sh, const V5Args &g, const RowTerms5 &t, int32_t mu,
                                           int32_t *__restrict__ ua, int32_t *__restrict__ ub) {
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int s = w >> 2, p = w & 3;
    const int L = tid & 63;
    const uint32_t q = s ? kQ1 : kQ0;
    for (int i = tid; i < kn; i += kV5Threads) {
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
    for (int k = tid; k < 2 * 27 * 64; k += kV5Threads) {
        (&sh.tsf[0][0][0])[k] = g.ts_f[k];
        (&sh.tsi[0][0][0])[k] = g.ts_i[k];
    }
    for (int k = tid; k < 2 * 16 * 64; k += kV5Threads) (&sh.tpost[0][0][0])[k] = g.tpost[k];
    __syncthreads();
    {
        const int e = (k2N - sh.barb) & (k2N - 1);
        for (int k = tid; k < kExt5; k += kV5Threads) {
            sh.E[0][k] = 0;
            sh.E[1][k] = ((k - e) & (k2N - 1)) < kN ? (uint32_t)mu : 0u - (uint32_t)mu;
        }
    }
    __syncthreads();
    const bool mac = p < 2;                 // wave (s, c = p): MAC + inverse for output c
    const int c_out = p;
    const int c_in = p >> 1, lvl = p & 1;   // digit poly p = 2 c_in + lvl
    uint32_t *sc = sh.scratch[w];
    uint4 bk[4][4];
    int inext = 0;
#ifdef TFHE_AMD_V5_STAMPS
    unsigned long long t_prev = __builtin_amdgcn_s_memtime();
#endif
    while (inext < kn && sh.bara[inext] == 0) ++inext;
    if (mac && inext < kn) load_bk(g, inext, s, c_out, L, bk);
    for (int i = inext; i < kn;) {
        const int a = sh.bara[i];
        int j = i + 1;                       // next non-trivial step (bara = 0: identity, :705)
        while (j < kn && sh.bara[j] == 0) ++j;
        // 1. decomposition of digit poly p (tgsw-functions.cu:300-413) + forward NTT
        uint32_t D[1][16];
        {
            const int base = (L - a) & (k2N - 1);
            const int sh_ = 22 - 10 * lvl;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const uint32_t tt = sh.E[c_in][base + 64 * r] - sh.E[c_in][L + 64 * r] + kDecompOffset;
                D[0][r] = ((tt >> sh_) & 1023u) + (q - 512u);
            }
        }
        const uint2 *tsf = &sh.tsf[s][0][L], *tsi = &sh.tsi[s][0][L], *tp = &sh.tpost[s][0][L];
        V5_STAMP(0);
        ntt_fwd<1>(D, sc, g.tu_f + 16 * s, tsf, L, q);
        store_C(sc, D[0], L);                                   // this wave's digit poly, NTT domain
        V5_STAMP(1);
        lds_barrier();                                          // B1: all digits in LDS
        V5_STAMP(2);
        uint32_t O[1][16];
        if (mac) {
            // 2. MAC for output c_out over 16 slots per lane (slot 16 L + r), REDC lazy
            const uint32_t qinv = s ? g.qinv_neg1 : g.qinv_neg0;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                lds_u32x4 dv[4];             // the 4 digit polys at slots 16 L + 4 v .. + 3
#pragma unroll
                for (int pp = 0; pp < 4; ++pp)
                    dv[pp] = reinterpret_cast<const lds_u32x4 *>(sh.scratch[4 * s + pp] + base_C(L))[v];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = 4 * v + e;
                    auto el = [&](const uint4 &x) { return e == 0 ? x.x : e == 1 ? x.y : e == 2 ? x.z : x.w; };
                    auto dl = [&](const lds_u32x4 &x) { return e == 0 ? x.x : e == 1 ? x.y : e == 2 ? x.z : x.w; };
                    const uint64_t x = (uint64_t)dl(dv[0]) * el(bk[0][v]) + (uint64_t)dl(dv[1]) * el(bk[1][v]) +
                                       (uint64_t)dl(dv[2]) * el(bk[2][v]) + (uint64_t)dl(dv[3]) * el(bk[3][v]);
                    const uint32_t m = (uint32_t)x * qinv;
                    O[0][r] = (uint32_t)((x + (uint64_t)m * q) >> 32);
                }
            }
            if (j < kn) load_bk(g, j, s, c_out, L, bk);         // next step's key, in flight
        }
        V5_STAMP(3);
        lds_barrier();                                          // B1b: digit polys consumed
        V5_STAMP(4);
        if (mac) {
            // 3. inverse NTT + post-twist (layout A: coefficient L + 64 r)
            ntt_inv_ct<1>(O, sc, g.tu_i + 16 * s, tsi, L, q);
            V5_STAMP(5);
            const uint32_t negq = 0u - q;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const uint2 tw = tp[r * 64];
                O[0][r] = shoup_lazy(O[0][r], tw.x, tw.y, negq);
            }
            // 4a. CRT give: wave (s, c) keeps r in [8 s, 8 s + 8), gives the other half
            if (s == 0) crt5_give<0>(sc, O[0], L);
            else crt5_give<1>(sc, O[0], L);
        }
        V5_STAMP(6);
        lds_barrier();                                          // B2 (uniform control flow)
        V5_STAMP(7);
        if (mac) {
            // 4b. CRT take + accumulate into E (both primes' residues of the kept half)
            if (s == 0) crt5_take<0>(sh, sh.scratch[w ^ 4], O[0], c_out, L, g);
            else crt5_take<1>(sh, sh.scratch[w ^ 4], O[0], c_out, L, g);
        }
        V5_STAMP(8);
        lds_barrier();                                          // B3: E updated
        V5_STAMP(9);
        i = j;
    }
    for (int j = tid; j < kN; j += kV5Threads) ua[j] = (int32_t)sh.E[0][(k2N - j) & (k2N - 1)];
    if (tid == 0) *ub = (int32_t)sh.E[1][0];
}

__global__ __launch_bounds__(kV5Threads, 1) void k_blind_rotate_v5(V5Args g, int B, BrInput in0, BrInput in1,
                                                                 int32_t mu, int32_t *__restrict__ u_a,
                                                                 int32_t *__restrict__ u_b) {
    __shared__ V5Shared sh;
    const int gct = blockIdx.x;
    const int half = gct >= B;
    const int idx = half ? gct - B : gct;
    const BrInput &in = half ? in1 : in0;
    RowTerms5 t;
    t.c = in.c; t.sa = in.sa; t.sb = in.sb; t.sc = 0;
    t.xa = in.x_a + (size_t)idx * kn; t.xb = in.x_b + idx;
    t.ya = in.sb ? in.y_a + (size_t)idx * kn : nullptr; t.yb = in.sb ? in.y_b + idx : nullptr;
    t.za = nullptr; t.zb = nullptr;
    br_v5_body(sh, g, t, mu, u_a + (size_t)gct * kN, u_b + gct);
}

__global__ __launch_bounds__(kV5Threads, 1) void k_blind_rotate_v5_rows(V5Args g, int B, const CircRow *__restrict__ rows,
                                                                      const int32_t *__restrict__ wa,
                                                                      const int32_t *__restrict__ wb, int32_t mu,
                                                                      int32_t *__restrict__ u_a,
                                                                      int32_t *__restrict__ u_b) {
    __shared__ V5Shared sh;
    const int k = blockIdx.x, r = blockIdx.y;
    const CircRow row = rows[r];
    auto wire = [&](int w, const int32_t *&pa, const int32_t *&pb) {
        if (w < 0) { pa = nullptr; pb = nullptr; return; }
        const size_t slot = (size_t)w * B + k;
        pa = wa + slot * kn;
        pb = wb + slot;
    };
    RowTerms5 t;
    t.c = row.c; t.sa = row.sa; t.sb = row.sb; t.sc = row.sc;
    wire(row.x, t.xa, t.xb);
    wire(row.y, t.ya, t.yb);
    wire(row.z, t.za, t.zb);
    const size_t slot = (size_t)r * B + k;
    br_v5_body(sh, g, t, mu, u_a + slot * kN, u_b + slot);
}

}  // namespace

static V5Args v5_args(const DeviceKey &key) {
    V5Args g;
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

#ifdef TFHE_AMD_V5_STAMPS
}  // namespace tfhe_amd
extern "C" int tfhe_amd_debug_v5_stamps(unsigned long long *out, int reset) {
    unsigned long long h[24];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(tfhe_amd::g_v5_stamps), sizeof h) != hipSuccess) return -2;
    for (int i = 0; i < 24; i++) out[i] = h[i];
    if (reset) {
        unsigned long long z[24] = {0};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(tfhe_amd::g_v5_stamps), z, sizeof z);
    }
    return 0;
}
namespace tfhe_amd {
#endif

hipError_t launch_blind_rotate_v5(const DeviceKey &key, int B, int halves, const BrInput *in, int32_t mu,
                                  int32_t *u_a, int32_t *u_b, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    const BrInput in1 = halves > 1 ? in[1] : in[0];
    hipLaunchKernelGGL(k_blind_rotate_v5, dim3(B * halves), dim3(kV5Threads), 0, s, v5_args(key), B, in[0], in1, mu,
                       u_a, u_b);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_v5_rows(const DeviceKey &key, int B, int nrows, const CircRow *rows, const int32_t *wa,
                                       const int32_t *wb, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t s) {
    if (B <= 0 || nrows <= 0) return hipSuccess;
    if (nrows > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_blind_rotate_v5_rows, dim3(B, nrows), dim3(kV5Threads), 0, s, v5_args(key), B, rows, wa, wb,
                       mu, u_a, u_b);
    return hipGetLastError();
}

}  // namespace tfhe_amd
