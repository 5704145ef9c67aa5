// bootstrap.hip — blind rotation (tfhe_blindRotate_FFT + extraction) on gfx950.
//
// Reference path replaced (gpuParallel/):
//   tfhe_bootstrap_woKS_FFT            lwe-bootstrapping-functions-fft.cu:1834-1870
//   tfhe_blindRotateAndExtract_FFT     :1408-1456
//   tfhe_blindRotate_FFT               :676-737   (skip bara_i == 0, :705)
//   tfhe_MuxRotate_FFT                 :105-185
//   tLweMulByXaiMinusOne               tlwe-functions.cu:334-349 -> toruspolynomial-functions.cu:191-235
//   tGswFFTExternMulToTLwe             tgsw-fft-operations.cu:124-264
//   tGswTorus32PolynomialDecompH       tgsw-functions.cu:300-413
//   tLweExtractLweSampleIndex(0)       lwe.cu:41-56
// and the reference GPU batch (comparator) bootstrapAndKeySwitch_n_Bit boot-gates.cu:2481-2629,
// which issues 2 500 launches per batch; here one launch runs all 500 CMux steps with the
// accumulator resident in LDS.
//
// v1 kernel: one 256-thread workgroup per ciphertext; the external product's 8 forward and
// 4 inverse negacyclic NTTs (2 primes) run as LDS-staged radix-2 stages.  The bootstrapping
// key (NTT domain, Montgomery form, 1/N folded) is read coalesced from HBM/L2 per step.
#include "engine.h"
#include "modarith.h"

namespace tfhe_amd {

namespace {

constexpr int kBrThreads = 256;

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

// inverse negacyclic NTT (GS), bit-reversed -> natural, no 1/N (folded into the key)
template <int NPOLY, int PRIME_SHIFT>
__device__ __forceinline__ void ntt_inv_lds(uint32_t *buf, const NttTables *__restrict__ tab) {
    const int tid = threadIdx.x;
    int logt = 0;
    for (int m = kN; m > 1; m >>= 1) {
        const int h = m >> 1;
        const int t = 1 << logt;
        for (int b = tid; b < NPOLY * (kN / 2); b += blockDim.x) {
            const int pi = b >> (kLogN - 1);
            const int k = b & (kN / 2 - 1);
            const int s = pi >> PRIME_SHIFT;
            const uint32_t q = q_of(s);
            const int blk = k >> logt;
            const int j = (blk << (logt + 1)) + (k & (t - 1));
            const uint32_t w = tab->ipsi[s][h + blk], wp = tab->ipsip[s][h + blk];
            uint32_t *x = buf + pi * kN;
            const uint32_t u = x[j], v = x[j + t];
            x[j] = add_mod(u, v, q);
            x[j + t] = mul_shoup(sub_mod(u, v, q), w, wp, q);
        }
        ++logt;
        __syncthreads();
    }
}

struct BrShared {
    uint32_t acc[2][kN];        // TLWE accumulator (a, b)
    uint32_t D[2][kKpl][kN];    // digit polys per prime (NTT domain after the forward pass)
    uint32_t O[2][2][kN];       // MAC outputs per prime
    int bara[512];
};

// one CMux step: acc <- ExtProd(BK_i, (X^a - 1) acc) + acc      (tfhe_MuxRotate_FFT)
__device__ __forceinline__ void cmux_step(BrShared &sh, const uint32_t *__restrict__ bki,
                                          const NttTables *__restrict__ tab, int a) {
    const int tid = threadIdx.x;
    // (X^a - 1) * acc  fused with the gadget decomposition (offset trick, tgsw-functions.cu:322-351)
    for (int idx = tid; idx < 2 * kN; idx += kBrThreads) {
        const int c = idx >> kLogN, j = idx & (kN - 1);
        const int si = (j - a) & (k2N - 1);
        const uint32_t r = si < kN ? sh.acc[c][si] : 0u - sh.acc[c][si - kN];
        const uint32_t v = r - sh.acc[c][j] + kDecompOffset;
        const int32_t d0 = (int32_t)((v >> 22) & 1023u) - 512;
        const int32_t d1 = (int32_t)((v >> 12) & 1023u) - 512;
        sh.D[0][2 * c + 0][j] = digit_mod(d0, kQ0);
        sh.D[1][2 * c + 0][j] = digit_mod(d0, kQ1);
        sh.D[0][2 * c + 1][j] = digit_mod(d1, kQ0);
        sh.D[1][2 * c + 1][j] = digit_mod(d1, kQ1);
    }
    __syncthreads();
    ntt_fwd_lds<2 * kKpl, 2>(&sh.D[0][0][0], tab, -1);
    // pointwise MAC with BK_i: O[s][c] = sum_p D[s][p] * BK_i[s][p][c]   (tLweFFTAddMulRTo)
    for (int idx = tid; idx < 4 * kN; idx += kBrThreads) {
        const int s = idx >> (kLogN + 1), c = (idx >> kLogN) & 1, j = idx & (kN - 1);
        const uint32_t *b = bki + ((size_t)(s * kKpl) * 2 + c) * kN + j;
        uint64_t accv = 0;
#pragma unroll
        for (int p = 0; p < kKpl; ++p) accv += (uint64_t)sh.D[s][p][j] * b[(size_t)p * 2 * kN];
        sh.O[s][c][j] = redc(accv, q_of(s), tab->qinv_neg[s]);
    }
    __syncthreads();
    ntt_inv_lds<4, 1>(&sh.O[0][0][0], tab);
    // back to the torus (exact) and accumulate (tLweAddTo)
    const uint32_t h = tab->crt_h, hp = tab->crt_hp;
    for (int idx = tid; idx < 2 * kN; idx += kBrThreads) {
        const int c = idx >> kLogN, j = idx & (kN - 1);
        sh.acc[c][j] += crt_torus(sh.O[0][c][j], sh.O[1][c][j], h, hp);
    }
    __syncthreads();
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
