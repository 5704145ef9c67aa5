// ntt_wave.h — register-resident negacyclic NTT building blocks shared by the blind-rotation
// kernels (blind_rotate_v4.hip; key layouts in ntt_key.hip).  One wave holds one 1024-point
// polynomial as 16 values per lane in three layouts
//   A: lane L, reg r <-> j = L + 64 r          (wave-uniform twiddles: SGPRs)
//   B: j = (L & 3) | r << 2 | (L >> 2) << 6
//   C: j = 16 L + r
// and moves between them with two LDS transposes per transform through a per-wave padded
// scratch (word address j + 4 (j >> 6): conflict-free for b32 A/B and b128 C accesses).
#pragma once
#include "engine.h"
#include "modarith.h"

namespace tfhe_amd {
namespace {

constexpr int kPadRow = kN + 64;   // padded scratch row: index j at word j + 4 (j >> 6)

// Timing diagnostics only (wrong results): TFHE_AMD_DIAG_TW reads every stream twiddle from
// slot 0, TFHE_AMD_DIAG_BK reads BK_0 at every step.
#ifdef TFHE_AMD_DIAG_TW
#define TW_SLOT(x) 0
#else
#define TW_SLOT(x) (x)
#endif

__device__ __forceinline__ uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }

// 16-B LDS vector that may alias the uint32_t view of the same scratch (the transposes write
// b32 and read b128 and vice versa: without may_alias, TBAA lets the compiler hoist the b128
// reads above the b32 writes of the same wave)
typedef uint32_t lds_u32x4 __attribute__((ext_vector_type(4), may_alias));

// Shoup product y * w mod q, lazy: [0, 2q) for any y < 2^32.  y*w - qh*q (mod 2^32) is
// folded into one v_mad_u64_u32: qh * (2^32 - q) + lo(y*w).
__device__ __forceinline__ uint32_t shoup_lazy(uint32_t y, uint32_t w, uint32_t wp, uint32_t negq) {
    const uint32_t qh = __umulhi(y, wp);
    return (uint32_t)((uint64_t)qh * negq + (uint32_t)(y * w));
}
// Cooley-Tukey (forward) butterfly WITHOUT reductions: inputs < B -> outputs < B + 2q.
// Digits enter < 2q, so after the 10 stages every value is < 22q < 2^32 (q < 2^27).
// The forward twiddle is stored NEGATED (wn = 2^32 - w, Shoup companion of w): then
// nt = qh q + lo(y wn) = -(y w - qh q) = -t (mod 2^32) with t in [0, 2q), one
// v_mad_u64_u32, and the two outputs are u - nt and u + nt + 2q (v_sub + v_add3): 5 VALU.
__device__ __forceinline__ void bf_ct(uint32_t &x, uint32_t &y, uint32_t wn, uint32_t wp, uint32_t q,
                                      uint32_t q2) {
    const uint32_t qh = __umulhi(y, wp);
    const uint32_t nt = (uint32_t)((uint64_t)qh * q + (uint32_t)(y * wn));
    const uint32_t u = x;
    x = u - nt;
    y = u + nt + q2;
}
// Gentleman-Sande (inverse) butterfly, Harvey: x, y in [0, 2q) -> [0, 2q)
__device__ __forceinline__ void bf_gs(uint32_t &x, uint32_t &y, uint32_t w, uint32_t wp, uint32_t negq,
                                      uint32_t q2) {
    const uint32_t s = x + y;
    const uint32_t t = x - y + q2;
    x = umin32(s, s - q2);
    y = shoup_lazy(t, w, wp, negq);
}

// Lanes of one wave exchange values through LDS in the transposes.  Single-thread
// semantics let the compiler hoist a lane's read above another lane's write whenever it
// can prove the two addresses differ FOR THE SAME LANE (it did, e.g. load_B(r < 8) above
// the last store_A: every coefficient came out wrong).  A wavefront-scope release/acquire
// pair around a wave barrier pins the order; LDS itself executes one wave's DS
// instructions in order.
__device__ __forceinline__ void wave_lds_sync() {
#ifdef TFHE_AMD_LDS_COMPILER_BARRIER
    asm volatile("" ::: "memory");      // experiment: rely on in-order LDS, compiler fence only
#else
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
}

// ---- layout transposes through the per-wave scratch (one polynomial)
__device__ __forceinline__ void store_A(uint32_t *sc, const uint32_t (&x)[16], int L) {
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[L + 68 * r] = x[r];            // j = L + 64 r
}
__device__ __forceinline__ void load_A(const uint32_t *sc, uint32_t (&x)[16], int L) {
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = sc[L + 68 * r];
}
__device__ __forceinline__ int base_B(int L) { return (L & 3) + 68 * (L >> 2); }
__device__ __forceinline__ void store_B(uint32_t *sc, const uint32_t (&x)[16], int L) {
    uint32_t *p = sc + base_B(L);
#pragma unroll
    for (int r = 0; r < 16; ++r) p[4 * r] = x[r];                   // j = (L&3) | r<<2 | (L>>2)<<6
}
__device__ __forceinline__ void load_B(const uint32_t *sc, uint32_t (&x)[16], int L) {
    const uint32_t *p = sc + base_B(L);
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = p[4 * r];
}
__device__ __forceinline__ int base_C(int L) { return 16 * L + 4 * (L >> 2); }
__device__ __forceinline__ void store_C(uint32_t *sc, const uint32_t (&x)[16], int L) {
    lds_u32x4 *p = reinterpret_cast<lds_u32x4 *>(sc + base_C(L));    // j = 16 L + r
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        lds_u32x4 t;
        t.x = x[4 * v]; t.y = x[4 * v + 1]; t.z = x[4 * v + 2]; t.w = x[4 * v + 3];
        p[v] = t;
    }
}
__device__ __forceinline__ void load_C(const uint32_t *sc, uint32_t (&x)[16], int L) {
    const lds_u32x4 *p = reinterpret_cast<const lds_u32x4 *>(sc + base_C(L));
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const lds_u32x4 t = p[v];
        x[4 * v] = t.x; x[4 * v + 1] = t.y; x[4 * v + 2] = t.z; x[4 * v + 3] = t.w;
    }
}

// stream twiddle `slot` for this lane: from the up-front copy (NP == 1) or loaded now
template <int NP>
__device__ __forceinline__ uint2 tw_slot(const uint2 (&tall)[NP == 1 ? 27 : 1], const uint2 *__restrict__ ts, int slot) {
    if constexpr (NP == 1) return tall[slot];
    else return ts[TW_SLOT(slot * 64)];
}

// ---- forward NTT of NP polys (layout A in, layout C out), values < 2q in, < 22q out
// (NP == 1, the latency kernel: all 27 stream twiddles are read at entry, before the layout-A
// stages and the transposes, so no stage group waits for its twiddle load)
template <int NP>
__device__ __forceinline__ void ntt_fwd(uint32_t (&x)[NP][16], uint32_t *sc, const uint2 *__restrict__ tu,
                                        const uint2 *__restrict__ ts, int L, uint32_t q) {
    const uint32_t q2 = 2 * q;
    uint2 tall[NP == 1 ? 27 : 1];
    if constexpr (NP == 1) {
#pragma unroll
        for (int g = 0; g < 27; ++g) tall[g] = ts[TW_SLOT(g * 64)];
    }
#pragma unroll
    for (int K = 9; K >= 6; --K) {                     // layout A, uniform twiddles
        const int d = 1 << (K - 6);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & d) continue;
            const uint2 t = tu[(1 << (9 - K)) + (r >> (K - 5))];
#pragma unroll
            for (int p = 0; p < NP; ++p) bf_ct(x[p][r], x[p][r + d], t.x, t.y, q, q2);
        }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        store_A(sc, x[p], L);
        wave_lds_sync();
        load_B(sc, x[p], L);
        wave_lds_sync();
    }
    int slot = 0;
#pragma unroll
    for (int K = 5; K >= 2; --K) {                     // layout B, per-lane twiddles
        const int d = 1 << (K - 2), cnt = 1 << (5 - K);
        uint2 tw[8];
#pragma unroll
        for (int g = 0; g < cnt; ++g) tw[g] = tw_slot<NP>(tall, ts, slot + g);
        slot += cnt;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & d) continue;
            const uint2 t = tw[r >> (K - 1)];
#pragma unroll
            for (int p = 0; p < NP; ++p) bf_ct(x[p][r], x[p][r + d], t.x, t.y, q, q2);
        }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        store_B(sc, x[p], L);
        wave_lds_sync();
        load_C(sc, x[p], L);
        wave_lds_sync();
    }
#pragma unroll
    for (int K = 1; K >= 0; --K) {                     // layout C
        const int d = 1 << K, cnt = 1 << (3 - K);
        uint2 tw[8];
#pragma unroll
        for (int g = 0; g < cnt; ++g) tw[g] = tw_slot<NP>(tall, ts, slot + g);
        slot += cnt;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & d) continue;
            const uint2 t = tw[r >> (K + 1)];
#pragma unroll
            for (int p = 0; p < NP; ++p) bf_ct(x[p][r], x[p][r + d], t.x, t.y, q, q2);
        }
    }
}

// ---- inverse NTT of NP polys (layout C in, layout A out), values [0,2q) -> [0,2q)
template <int NP>
__device__ __forceinline__ void ntt_inv(uint32_t (&x)[NP][16], uint32_t *sc, const uint2 *__restrict__ tu,
                                        const uint2 *__restrict__ ts, int L, uint32_t q) {
    const uint32_t q2 = 2 * q, negq = 0u - q;
    int slot = 0;
#pragma unroll
    for (int K = 0; K <= 3; ++K) {                     // layout C
        const int d = 1 << K, cnt = 1 << (3 - K);
        uint2 tw[8];
#pragma unroll
        for (int g = 0; g < cnt; ++g) tw[g] = ts[TW_SLOT((slot + g) * 64)];
        slot += cnt;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & d) continue;
            const uint2 t = tw[r >> (K + 1)];
#pragma unroll
            for (int p = 0; p < NP; ++p) bf_gs(x[p][r], x[p][r + d], t.x, t.y, negq, q2);
        }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        store_C(sc, x[p], L);
        wave_lds_sync();
        load_B(sc, x[p], L);
        wave_lds_sync();
    }
#pragma unroll
    for (int K = 4; K <= 5; ++K) {                     // layout B
        const int d = 1 << (K - 2), cnt = 1 << (5 - K);
        uint2 tw[2];
#pragma unroll
        for (int g = 0; g < cnt; ++g) tw[g] = ts[TW_SLOT((slot + g) * 64)];
        slot += cnt;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & d) continue;
            const uint2 t = tw[r >> (K - 1)];
#pragma unroll
            for (int p = 0; p < NP; ++p) bf_gs(x[p][r], x[p][r + d], t.x, t.y, negq, q2);
        }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        store_B(sc, x[p], L);
        wave_lds_sync();
        load_A(sc, x[p], L);
        wave_lds_sync();
    }
#pragma unroll
    for (int K = 6; K <= 9; ++K) {                     // layout A, uniform twiddles
        const int d = 1 << (K - 6);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & d) continue;
            const uint2 t = tu[(1 << (9 - K)) + (r >> (K - 5))];
#pragma unroll
            for (int p = 0; p < NP; ++p) bf_gs(x[p][r], x[p][r + d], t.x, t.y, negq, q2);
        }
    }
}

// ---- inverse NTT as a Cooley-Tukey DIT transform of NP polys: bit-reversed slots in
// layout C (k = 16 L + r), natural order out in layout A, values < 3.75q in -> < 31.75q out
// (no reductions; the caller applies the psi^-n post-twist).  Stage s pairs k, k + 2^s with
// twiddle psi^-(p 2^(10-s)), p = k mod 2^s:
//   C, s = 0..3: p = r mod 2^s            -> wave-uniform, tu[(2^s - 1) + p]
//   B, s = 4, 5: p = (L & 3) | g << 2     -> stream slots g = r mod 2^(s-2)   (4 + 8)
//   A, s = 6..9: p = L + 64 g             -> stream slots g = r mod 2^(s-6)   (1 + 2 + 4 + 8)
// Twiddles are stored negated (bf_ct).  27 stream slots in consumption order.
template <int NP>
__device__ __forceinline__ void ntt_inv_ct(uint32_t (&x)[NP][16], uint32_t *sc, const uint2 *__restrict__ tu,
                                           const uint2 *__restrict__ ts, int L, uint32_t q) {
    const uint32_t q2 = 2 * q;
    uint2 tall[NP == 1 ? 27 : 1];                      // NP == 1: all stream twiddles up front
    if constexpr (NP == 1) {
#pragma unroll
        for (int g = 0; g < 27; ++g) tall[g] = ts[TW_SLOT(g * 64)];
    }
#pragma unroll
    for (int S = 0; S <= 3; ++S) {                     // layout C, uniform twiddles
        const int d = 1 << S;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & d) continue;
            if (S <= 1 && (r & (d - 1)) == 0) {
                // p = 0: twiddle 1, no multiply.  Bounds: < 3.75q in; after stage 0 < 7.75q
                // (K = 4q), after stage 1 < 15.75q (K = 8q); the 8 Shoup stages after it
                // add 2q each: < 31.75q < 2^32 (q < 2^27)
                const uint32_t K = S == 0 ? 4 * q : 8 * q;
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    const uint32_t u = x[p][r], v = x[p][r + d];
                    x[p][r] = u + v;
                    x[p][r + d] = u + K - v;
                }
                continue;
            }
            const uint2 t = tu[(d - 1) + (r & (d - 1))];
#pragma unroll
            for (int p = 0; p < NP; ++p) bf_ct(x[p][r], x[p][r + d], t.x, t.y, q, q2);
        }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        store_C(sc, x[p], L);
        wave_lds_sync();
        load_B(sc, x[p], L);
        wave_lds_sync();
    }
    int slot = 0;
#pragma unroll
    for (int S = 4; S <= 5; ++S) {                     // layout B
        const int d = 1 << (S - 2);
        uint2 tw[8];
#pragma unroll
        for (int g = 0; g < d; ++g) tw[g] = tw_slot<NP>(tall, ts, slot + g);
        slot += d;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & d) continue;
            const uint2 t = tw[r & (d - 1)];
#pragma unroll
            for (int p = 0; p < NP; ++p) bf_ct(x[p][r], x[p][r + d], t.x, t.y, q, q2);
        }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        store_B(sc, x[p], L);
        wave_lds_sync();
        load_A(sc, x[p], L);
        wave_lds_sync();
    }
#pragma unroll
    for (int S = 6; S <= 9; ++S) {                     // layout A
        const int d = 1 << (S - 6);
        uint2 tw[8];
#pragma unroll
        for (int g = 0; g < d; ++g) tw[g] = tw_slot<NP>(tall, ts, slot + g);
        slot += d;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & d) continue;
            const uint2 t = tw[r & (d - 1)];
#pragma unroll
            for (int p = 0; p < NP; ++p) bf_ct(x[p][r], x[p][r + d], t.x, t.y, q, q2);
        }
    }
}

}  // namespace
}  // namespace tfhe_amd
