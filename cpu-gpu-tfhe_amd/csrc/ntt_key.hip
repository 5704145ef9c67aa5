// ntt_key.hip — the exact NTT kernels' key layout and twiddle streams (blind_rotate_v4.hip).
//
// The bootstrapping key in the NTT domain (two 27-bit primes, Montgomery form, 1/N folded; built
// by bootstrap.hip's k_bk_to_ntt in the coefficient layout [kn][2 primes][4 rows][2 c][N]) is
// re-laid out for the exact kernels' MAC: [kn][2 primes][2 c][4 rows][4 v][64 lanes][4 e], so
// that each lane's 16-B load holds the 4 consecutive coefficients 16 L + 4 v + e of its layout-C
// registers.  The twiddle streams are consumed in order by ntt_wave.h's transforms.
// (This file held the round-1 v2 blind rotation; its kernel is retired, the key layout and
// twiddles it introduced are what v4 reads.)
#include "engine.h"
#include "modarith.h"
#include "ntt_wave.h"

namespace tfhe_amd {

namespace {

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

// Twiddle tables of the exact kernels (v4), generated on the host in their consumption order:
// uniform forward / inverse [2 primes][16], then the per-lane streams [2][27][64] (forward) and
// [2][18][64] (inverse).
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

hipError_t launch_bk_v1_to_v2(const uint32_t *d_v1, uint32_t *d_v2, hipStream_t s) {
    hipLaunchKernelGGL(k_bk_v1_to_v2, dim3(kn * 2 * 8), dim3(256), 0, s, d_v1, d_v2);
    return hipGetLastError();
}

}  // namespace tfhe_amd
