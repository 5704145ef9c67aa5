/*
 * tfhe_core.h — core types of the TFHE C API, layout-compatible with the reference.
 * Replaces gpuParallel/tfhe_core.h:11-16 (EXPORT), :28 (Torus32) and the forward
 * declarations that cpuParallel's Cipher.h:7-8 pulls in through <tfhe/tfhe.h>.
 */
#ifndef TFHE_AMD_TFHE_CORE_H
#define TFHE_AMD_TFHE_CORE_H

#include <stdint.h>

#ifdef __cplusplus
#define EXPORT extern "C"
#else
#define EXPORT
#endif

typedef int32_t Torus32;   /* tfhe_core.h:28 */

struct LweParams;
struct LweKey;
struct LweSample;
struct LweKeySwitchKey;
struct TLweParams;
struct TLweKey;
struct TLweSample;
struct TLweSampleFFT;
struct TGswParams;
struct TGswKey;
struct TGswSample;
struct TGswSampleFFT;
struct LweBootstrappingKey;
struct LweBootstrappingKeyFFT;
struct IntPolynomial;
struct TorusPolynomial;
struct LagrangeHalfCPolynomial;
struct TFheGateBootstrappingParameterSet;
struct TFheGateBootstrappingCloudKeySet;
struct TFheGateBootstrappingSecretKeySet;

#ifndef __cplusplus
typedef struct LweParams LweParams;
typedef struct LweKey LweKey;
typedef struct LweSample LweSample;
typedef struct LweKeySwitchKey LweKeySwitchKey;
typedef struct TLweParams TLweParams;
typedef struct TLweKey TLweKey;
typedef struct TLweSample TLweSample;
typedef struct TLweSampleFFT TLweSampleFFT;
typedef struct TGswParams TGswParams;
typedef struct TGswKey TGswKey;
typedef struct TGswSample TGswSample;
typedef struct TGswSampleFFT TGswSampleFFT;
typedef struct LweBootstrappingKey LweBootstrappingKey;
typedef struct LweBootstrappingKeyFFT LweBootstrappingKeyFFT;
typedef struct IntPolynomial IntPolynomial;
typedef struct TorusPolynomial TorusPolynomial;
typedef struct LagrangeHalfCPolynomial LagrangeHalfCPolynomial;
typedef struct TFheGateBootstrappingParameterSet TFheGateBootstrappingParameterSet;
typedef struct TFheGateBootstrappingCloudKeySet TFheGateBootstrappingCloudKeySet;
typedef struct TFheGateBootstrappingSecretKeySet TFheGateBootstrappingSecretKeySet;
#endif

/* tfhe_gate_bootstrapping.cu:11-15: prints and aborts */
EXPORT void die_dramatically(const char *message);

#endif
