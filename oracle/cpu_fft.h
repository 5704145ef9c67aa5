/*
 * cpu_fft.h — TEST INFRASTRUCTURE ONLY: the optimized CPU baseline (double-precision FFT
 * external product, OpenMP over gates), timed by bench.py's cpu_baseline leg and checked
 * bit-exactly against the exact oracle (tfhe_oracle.h) by tests/test_cpu_baseline.py.
 * Layouts as in tfhe_oracle.h (BK int32 [500][4][2][1024], KSK int32 [1024][8][4][501]).
 */
#ifndef TFHE_CPU_FFT_H
#define TFHE_CPU_FFT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct CpuFftKey CpuFftKey;
/* pre-transforms the bootstrapping key (32.8 MB); borrows ksk (caller keeps it alive) */
CpuFftKey *cpufft_key_create(const int32_t *bk, const int32_t *ksk);
void cpufft_key_free(CpuFftKey *key);
/* largest |c - rint(c)| of any rounded external-product coefficient so far */
double cpufft_max_round_error(const CpuFftKey *key);

/* B gates res = KS(bootstrap((0, c) + sa ca + sb cb)), mu = 1/8 (boot-gates.cu:98-397) */
void cpufft_gate_batch(int B, int32_t c, int32_t sa, int32_t sb, int32_t *res_a, int32_t *res_b,
                       const int32_t *ca_a, const int32_t *ca_b, const int32_t *cb_a, const int32_t *cb_b,
                       const CpuFftKey *key, int nthreads);
/* B woKS bootstraps x (n = 500) -> u (N = 1024) */
void cpufft_woks_batch(int B, int32_t *out_a, int32_t *out_b, const CpuFftKey *key, int32_t mu,
                       const int32_t *x_a, const int32_t *x_b, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
