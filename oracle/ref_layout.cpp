// ref_layout.cpp — TEST INFRASTRUCTURE ONLY.  Prints sizeof/offsetof of the TFHE structs the
// C ABI must match, compiled against the REFERENCE headers in place (gpuParallel/*.h), as JSON.
// Used by tests/golden/make_golden.py -> tests/golden/abi_layout.json; tests/test_abi.py builds it
// with -DTFHE_AMD_HEADERS against include/ and compares.
#include <cstddef>
#include <cstdio>
#ifdef TFHE_AMD_HEADERS          // the same program against OUR include/ (tests/test_abi.py)
#include "tfhe/tfhe.h"
#else
#include "tfhe_core.h"
#include "lweparams.h"
#include "lwesamples.h"
#include "lwekey.h"
#include "lwekeyswitch.h"
#include "polynomials.h"
#include "tlwe.h"
#include "tgsw.h"
#include "lwebootstrappingkey.h"
#include "tfhe_gate_bootstrapping_structures.h"
#endif

#define F(S, f) printf("  \"%s.%s\": %zu,\n", #S, #f, offsetof(S, f))
#define Z(S) printf("  \"sizeof(%s)\": %zu,\n", #S, sizeof(S))

int main() {
    printf("{\n");
    Z(LweParams); F(LweParams, n); F(LweParams, alpha_min); F(LweParams, alpha_max);
    Z(TLweParams); F(TLweParams, N); F(TLweParams, k); F(TLweParams, alpha_min); F(TLweParams, alpha_max);
    F(TLweParams, extracted_lweparams);
    Z(TGswParams); F(TGswParams, l); F(TGswParams, Bgbit); F(TGswParams, Bg); F(TGswParams, halfBg);
    F(TGswParams, maskMod); F(TGswParams, tlwe_params); F(TGswParams, kpl); F(TGswParams, h); F(TGswParams, offset);
    Z(IntPolynomial); F(IntPolynomial, N); F(IntPolynomial, coefs);
    Z(TorusPolynomial); F(TorusPolynomial, N); F(TorusPolynomial, coefsT);
    Z(LweSample); F(LweSample, a); F(LweSample, b); F(LweSample, current_variance);
    Z(LweKey); F(LweKey, params); F(LweKey, key);
    Z(TLweKey); F(TLweKey, params); F(TLweKey, key);
    Z(TLweSample); F(TLweSample, a); F(TLweSample, b); F(TLweSample, current_variance); F(TLweSample, k);
    Z(TGswKey); F(TGswKey, params); F(TGswKey, tlwe_params); F(TGswKey, key); F(TGswKey, tlwe_key);
    Z(TGswSample); F(TGswSample, all_sample); F(TGswSample, bloc_sample); F(TGswSample, k); F(TGswSample, l);
    Z(TGswSampleFFT); F(TGswSampleFFT, all_samples); F(TGswSampleFFT, sample); F(TGswSampleFFT, k);
    F(TGswSampleFFT, l);
    Z(LweKeySwitchKey); F(LweKeySwitchKey, n); F(LweKeySwitchKey, t); F(LweKeySwitchKey, basebit);
    F(LweKeySwitchKey, base); F(LweKeySwitchKey, out_params); F(LweKeySwitchKey, ks0_raw);
    F(LweKeySwitchKey, ks1_raw); F(LweKeySwitchKey, ks);
    Z(LweBootstrappingKey); F(LweBootstrappingKey, in_out_params); F(LweBootstrappingKey, bk_params);
    F(LweBootstrappingKey, accum_params); F(LweBootstrappingKey, extract_params); F(LweBootstrappingKey, bk);
    F(LweBootstrappingKey, ks);
    Z(LweBootstrappingKeyFFT); F(LweBootstrappingKeyFFT, in_out_params); F(LweBootstrappingKeyFFT, bk_params);
    F(LweBootstrappingKeyFFT, accum_params); F(LweBootstrappingKeyFFT, extract_params);
    F(LweBootstrappingKeyFFT, bkFFT); F(LweBootstrappingKeyFFT, ks);
    Z(TFheGateBootstrappingParameterSet); F(TFheGateBootstrappingParameterSet, ks_t);
    F(TFheGateBootstrappingParameterSet, ks_basebit); F(TFheGateBootstrappingParameterSet, in_out_params);
    F(TFheGateBootstrappingParameterSet, tgsw_params);
    Z(TFheGateBootstrappingCloudKeySet); F(TFheGateBootstrappingCloudKeySet, params);
    F(TFheGateBootstrappingCloudKeySet, bk); F(TFheGateBootstrappingCloudKeySet, bkFFT);
    Z(TFheGateBootstrappingSecretKeySet); F(TFheGateBootstrappingSecretKeySet, params);
    F(TFheGateBootstrappingSecretKeySet, lwe_key); F(TFheGateBootstrappingSecretKeySet, tgsw_key);
    F(TFheGateBootstrappingSecretKeySet, cloud);
    printf("  \"_end\": 0\n}\n");
    return 0;
}
