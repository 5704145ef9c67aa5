// bootstrap.hip — the bootstrapping key's conversion to the exact NTT domain (device side of
// init_LweBootstrappingKeyFFT, lwe-bootstrapping-functions-fft.cu:60-89, for the exact kernels).
//
// Each coefficient-domain key polynomial (TGSW rows of bk_i, [kn][kKpl rows][2 c][N] int32) is
// reduced mod each of the two 27-bit primes and transformed by a forward negacyclic NTT (CT,
// twist merged into the twiddles), then scaled by N^-1 in Montgomery form, so that the exact
// kernels' MAC + REDC yields the product directly.  Output layout [i][prime][row][c][N];
// ntt_key.hip re-lays it out for blind_rotate_v4.hip's register layout.  (The round-1 v1 blind
// rotation that lived here, LDS-staged radix-2 stages, is retired.)
#include "engine.h"
#include "modarith.h"

namespace tfhe_amd {

namespace {

// forward negacyclic NTT (CT, merged twist) on NPOLY LDS-resident polys buf[pi][kN];
// the prime of poly pi is (sfix >= 0 ? sfix : pi >> PRIME_SHIFT).
template <int NPOLY, int PRIME_SHIFT>
__device__ __forceinline__ void ntt_fwd_lds(uint32_t *buf, const NttTables *__restrict__ tab, int sfix) {
    const int tid = threadIdx.x;
    int logt = kLogN;
    for (int m = 1; m < kN; m <<= 1) {
        --logt;
        const int t = 1 << logt;
        for (int b = tid; b < NPOLY * (kN / 2); b += blockDim.x) {
            const int pi = b >> (kLogN - 1);
            const int k = b & (kN / 2 - 1);
            const int s = sfix >= 0 ? sfix : (pi >> PRIME_SHIFT);
            const uint32_t q = q_of(s);
            const int blk = k >> logt;
            const int j = (blk << (logt + 1)) + (k & (t - 1));
            const uint32_t w = tab->psi[s][m + blk], wp = tab->psip[s][m + blk];
            uint32_t *x = buf + pi * kN;
            const uint32_t u = x[j];
            const uint32_t v = mul_shoup(x[j + t], w, wp, q);
            x[j] = add_mod(u, v, q);
            x[j + t] = sub_mod(u, v, q);
        }
        __syncthreads();
    }
}

// coefficient-domain BK -> NTT domain (Montgomery, 1/N folded): one workgroup per polynomial.
// Output layout [i][s][p][c][kN]  (analogue of init_LweBootstrappingKeyFFT :60-89).
__global__ __launch_bounds__(256) void k_bk_to_ntt(const int32_t *__restrict__ bk_coef,
                                                   uint32_t *__restrict__ bk_ntt,
                                                   const NttTables *__restrict__ tab) {
    __shared__ uint32_t buf[kN];
    const int poly = blockIdx.x;            // ((i * 2 + s) * 4 + p) * 2 + c
    const int c = poly & 1, p = (poly >> 1) & 3, s = (poly >> 3) & 1, i = poly >> 4;
    const uint32_t q = q_of(s);
    const int32_t *src = bk_coef + ((size_t)(i * kKpl + p) * 2 + c) * kN;
    for (int j = threadIdx.x; j < kN; j += blockDim.x) {
        const int64_t v = src[j];
        int64_t r = v % (int64_t)q;
        buf[j] = (uint32_t)(r < 0 ? r + q : r);
    }
    __syncthreads();
    ntt_fwd_lds<1, 0>(buf, tab, s);
    uint32_t *dst = bk_ntt + (size_t)poly * kN;
    for (int j = threadIdx.x; j < kN; j += blockDim.x)
        dst[j] = mul_shoup(buf[j], tab->bk_scale[s], tab->bk_scalep[s], q);
}

}  // namespace

hipError_t launch_bk_to_ntt(const int32_t *d_bk_coef, uint32_t *d_bk_ntt, const NttTables *d_tab,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_bk_to_ntt, dim3(kn * 2 * kKpl * 2), dim3(256), 0, s, d_bk_coef, d_bk_ntt, d_tab);
    return hipGetLastError();
}


}  // namespace tfhe_amd
