/*
 * tfhe.h — the TFHE C API this library exports, as a drop-in for the libtfhe that
 * cpuParallel/Cipher.cpp and cpuParallel/cloud.cpp link (compile.sh:1-2, Cipher.h:7-8).
 *
 * Struct layouts match the reference field-for-field (so code that dereferences
 * bk->params->in_out_params->n, bk->bkFFT->ks, ... keeps working):
 *   LweParams           gpuParallel/lweparams.h:13-28
 *   TLweParams          tlwe.h:10-28          TLweKey / TLweSample   tlwe.h:30-63
 *   TGswParams          tgsw.h:10-32          TGswKey / TGswSample   tgsw.h:35-76
 *   IntPolynomial, TorusPolynomial            polynomials.h:10-32
 *   LweSample           lwesamples.h:18-29    LweKey                 lwekey.h:10-20
 *   LweKeySwitchKey     lwekeyswitch.h:11-28
 *   LweBootstrappingKey(FFT)                  lwebootstrappingkey.h:10-59
 *   TFheGateBootstrapping{ParameterSet,CloudKeySet,SecretKeySet}
 *                                             tfhe_gate_bootstrapping_structures.h:9-63
 *   TGswSampleFFT       tgsw.h:78-96 (so that bk->bkFFT->bkFFT + i indexes the key's array)
 * TLweSampleFFT stays opaque (all_samples / sample are null): this engine keeps the
 * bootstrapping key on the GPU in its own transform layouts (fp64 FFT for the default kernel,
 * exact NTT for the guard's recomputation and the L1 entry points) instead of the reference's
 * LagrangeHalfC one; a TGswSampleFFT of a key is a handle the L1 functions map back to it.
 *
 * Semantics: synchronous, single-sample, reentrant (safe to call from
 * OpenMP threads as Cipher.cpp:116-120 does); result may alias an input; fatal errors
 * abort through die_dramatically like the reference.
 */
#ifndef TFHE_AMD_TFHE_H
#define TFHE_AMD_TFHE_H

#include "tfhe_core.h"
#include "tfhe_io.h"      /* the reference tfhe.h includes it too (gpuParallel/tfhe.h:26) */
#ifdef __cplusplus
#include <cmath>          /* callers rely on it arriving via tfhe.h -> numeric_functions.h:10
                             (<random>); cloud.cpp:43 calls pow() without including it */
#endif

struct LweParams {
    const int n;
    const double alpha_min;
    const double alpha_max;
};

struct TLweParams {
    const int N;
    const int k;
    const double alpha_min;
    const double alpha_max;
    const struct LweParams extracted_lweparams;
};

struct TGswParams {
    const int l;
    const int Bgbit;
    const int Bg;
    const int32_t halfBg;
    const uint32_t maskMod;
    const struct TLweParams *tlwe_params;
    const int kpl;
    Torus32 *h;
    uint32_t offset;
};

struct IntPolynomial {
    const int N;
    int *coefs;
};

struct TorusPolynomial {
    const int N;
    Torus32 *coefsT;
};

struct LweSample {
    Torus32 *a;
    Torus32 b;
    double current_variance;
};

struct LweKey {
    const struct LweParams *params;
    int *key;
};

struct TLweKey {
    const struct TLweParams *params;
    struct IntPolynomial *key;
};

struct TLweSample {
    struct TorusPolynomial *a;
    struct TorusPolynomial *b;
    double current_variance;
    const int k;
};

struct TGswKey {
    const struct TGswParams *params;
    const struct TLweParams *tlwe_params;
    struct IntPolynomial *key;
    struct TLweKey tlwe_key;
};

struct TGswSample {
    struct TLweSample *all_sample;
    struct TLweSample **bloc_sample;
    const int k;
    const int l;
};

struct TGswSampleFFT {
    struct TLweSampleFFT *all_samples;
    struct TLweSampleFFT **sample;
    const int k;
    const int l;
};

struct LweKeySwitchKey {
    int n;
    int t;
    int basebit;
    int base;
    const struct LweParams *out_params;
    struct LweSample *ks0_raw;
    struct LweSample **ks1_raw;
    struct LweSample ***ks;
};

struct LweBootstrappingKey {
    const struct LweParams *in_out_params;
    const struct TGswParams *bk_params;
    const struct TLweParams *accum_params;
    const struct LweParams *extract_params;
    struct TGswSample *bk;
    struct LweKeySwitchKey *ks;
};

struct LweBootstrappingKeyFFT {
    const struct LweParams *in_out_params;
    const struct TGswParams *bk_params;
    const struct TLweParams *accum_params;
    const struct LweParams *extract_params;
    const struct TGswSampleFFT *bkFFT;
    const struct LweKeySwitchKey *ks;
};

struct TFheGateBootstrappingParameterSet {
    const int ks_t;
    const int ks_basebit;
    const struct LweParams *const in_out_params;
    const struct TGswParams *const tgsw_params;
};

struct TFheGateBootstrappingCloudKeySet {
    const struct TFheGateBootstrappingParameterSet *const params;
    const struct LweBootstrappingKey *const bk;
    const struct LweBootstrappingKeyFFT *const bkFFT;
};

struct TFheGateBootstrappingSecretKeySet {
    const struct TFheGateBootstrappingParameterSet *params;
    const struct LweKey *lwe_key;
    const struct TGswKey *tgsw_key;
    const struct TFheGateBootstrappingCloudKeySet cloud;
};

/* ---------------------------------------------------------------- numerics */
/* numeric-functions.cu:16-19, 22-28, 33-40, 46-77 */
EXPORT void tfhe_random_generator_setSeed(uint32_t *values, int size);
EXPORT Torus32 dtot32(double d);
EXPORT double t32tod(Torus32 x);
EXPORT Torus32 gaussian32(Torus32 message, double sigma);
EXPORT Torus32 approxPhase(Torus32 phase, int Msize);
EXPORT int modSwitchFromTorus32(Torus32 phase, int Msize);
EXPORT Torus32 modSwitchToTorus32(int mu, int Msize);

/* ------------------------------------------------------ parameters and keys */
/* tfhe_gate_bootstrapping.cu:25-125 */
EXPORT TFheGateBootstrappingParameterSet *new_default_gate_bootstrapping_parameters(int minimum_lambda);
EXPORT void delete_gate_bootstrapping_parameters(TFheGateBootstrappingParameterSet *params);
EXPORT TFheGateBootstrappingSecretKeySet *
new_random_gate_bootstrapping_secret_keyset(const TFheGateBootstrappingParameterSet *params);
EXPORT void delete_gate_bootstrapping_secret_keyset(TFheGateBootstrappingSecretKeySet *keyset);
EXPORT void delete_gate_bootstrapping_cloud_keyset(TFheGateBootstrappingCloudKeySet *keyset);
EXPORT LweSample *new_gate_bootstrapping_ciphertext(const TFheGateBootstrappingParameterSet *params);
EXPORT LweSample *new_gate_bootstrapping_ciphertext_array(int nbelems, const TFheGateBootstrappingParameterSet *params);
EXPORT void delete_gate_bootstrapping_ciphertext(LweSample *sample);
EXPORT void delete_gate_bootstrapping_ciphertext_array(int nbelems, LweSample *samples);
EXPORT void bootsSymEncrypt(LweSample *result, int message, const TFheGateBootstrappingSecretKeySet *key);
EXPORT int bootsSymDecrypt(const LweSample *sample, const TFheGateBootstrappingSecretKeySet *key);

/* ------------------------------------------------------------- LWE samples */
/* lwesamples.h / lwe-functions.cu:21-291 */
EXPORT LweSample *new_LweSample(const LweParams *params);
EXPORT LweSample *new_LweSample_array(int nbelts, const LweParams *params);
EXPORT void delete_LweSample(LweSample *obj);
EXPORT void delete_LweSample_array(int nbelts, LweSample *obj);
EXPORT void lweKeyGen(LweKey *result);
EXPORT void lweSymEncrypt(LweSample *result, Torus32 message, double alpha, const LweKey *key);
EXPORT void lweSymEncryptWithExternalNoise(LweSample *result, Torus32 message, double noise, double alpha,
                                           const LweKey *key);
EXPORT Torus32 lwePhase(const LweSample *sample, const LweKey *key);
EXPORT Torus32 lweSymDecrypt(const LweSample *sample, const LweKey *key, const int Msize);
EXPORT void lweClear(LweSample *result, const LweParams *params);
EXPORT void lweCopy(LweSample *result, const LweSample *sample, const LweParams *params);
EXPORT void lweNegate(LweSample *result, const LweSample *sample, const LweParams *params);
EXPORT void lweNoiselessTrivial(LweSample *result, Torus32 mu, const LweParams *params);
EXPORT void lweAddTo(LweSample *result, const LweSample *sample, const LweParams *params);
EXPORT void lweSubTo(LweSample *result, const LweSample *sample, const LweParams *params);
EXPORT void lweAddMulTo(LweSample *result, int p, const LweSample *sample, const LweParams *params);
EXPORT void lweSubMulTo(LweSample *result, int p, const LweSample *sample, const LweParams *params);

/* ------------------------------------------------------- bootstrapping core */
/* lwe-bootstrapping-functions-fft.cu:1834-1870 (woKS, result has dimension N=1024),
 * :1884-1910 (with key switch); lwe-keyswitch-functions.cu:955-987 */
EXPORT void tfhe_bootstrap_woKS_FFT(LweSample *result, const LweBootstrappingKeyFFT *bk, Torus32 mu,
                                    const LweSample *x);
EXPORT void tfhe_bootstrap_FFT(LweSample *result, const LweBootstrappingKeyFFT *bk, Torus32 mu,
                               const LweSample *x);
EXPORT void lweKeySwitch(LweSample *result, const LweKeySwitchKey *ks, const LweSample *sample);

/* L1 (tfhe.h:42-43: lwe-bootstrapping-functions-fft.cu:676-737, 1408-1456; tgsw_functions.h:70:
 * tgsw-fft-operations.cu:124-264).  bk / gsw: an element of a key's array bk->bkFFT->bkFFT (the
 * loop uses bk + i for step i < n).  Exact products (the reference's FFT truncates its double
 * result, fft_processor_fftw.cu:177: see DESIGN.md §2). */
EXPORT void tfhe_blindRotate_FFT(TLweSample *accum, const TGswSampleFFT *bk, const int *bara, const int n,
                                 const TGswParams *bk_params);
EXPORT void tfhe_blindRotateAndExtract_FFT(LweSample *result, const TorusPolynomial *v, const TGswSampleFFT *bk,
                                           const int barb, const int *bara, const int n, const TGswParams *bk_params);
EXPORT void tGswFFTExternMulToTLwe(TLweSample *accum, const TGswSampleFFT *gsw, const TGswParams *params);
/* tlwe.h:222-231, polynomials.h:97-102 */
EXPORT TLweSample *new_TLweSample(const TLweParams *params);
EXPORT void delete_TLweSample(TLweSample *obj);
EXPORT TorusPolynomial *new_TorusPolynomial(const int N);
EXPORT void delete_TorusPolynomial(TorusPolynomial *obj);

/* ---------------------------------------------------------------- gates */
/* tfhe_gate_bootstrapping_functions.h:48-89; boot-gates.cu:98-448 */
EXPORT void bootsNAND(LweSample *result, const LweSample *ca, const LweSample *cb, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsOR(LweSample *result, const LweSample *ca, const LweSample *cb, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsAND(LweSample *result, const LweSample *ca, const LweSample *cb, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsXOR(LweSample *result, const LweSample *ca, const LweSample *cb, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsXNOR(LweSample *result, const LweSample *ca, const LweSample *cb, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsNOR(LweSample *result, const LweSample *ca, const LweSample *cb, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsANDNY(LweSample *result, const LweSample *ca, const LweSample *cb, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsANDYN(LweSample *result, const LweSample *ca, const LweSample *cb, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsORNY(LweSample *result, const LweSample *ca, const LweSample *cb, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsORYN(LweSample *result, const LweSample *ca, const LweSample *cb, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsNOT(LweSample *result, const LweSample *ca, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsCOPY(LweSample *result, const LweSample *ca, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsCONSTANT(LweSample *result, int value, const TFheGateBootstrappingCloudKeySet *bk);
EXPORT void bootsMUX(LweSample *result, const LweSample *a, const LweSample *b, const LweSample *c,
                     const TFheGateBootstrappingCloudKeySet *bk);

#endif
