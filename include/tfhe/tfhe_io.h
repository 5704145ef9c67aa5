/*
 * tfhe_io.h — key / ciphertext serialisation, byte-compatible with the reference's
 * gpuParallel/tfhe_io.cu (and tfhe_generic_streams.cu for the text headers), so files
 * written by either library are read by the other.
 *
 * Provided: the gate-bootstrapping entry points cpuParallel/main.cpp:26-33,66-71 and
 * cloud.cpp:138-161 / Cipher.cpp:18-20 call, plus the LWE-sample ones they forward to.
 *   export_/new_tfheGateBootstrappingParameterSet_*   tfhe_io.h:379-399 (tfhe_io.cu:1014-1078)
 *   export_/new_tfheGateBootstrappingCloudKeySet_*    tfhe_io.h:410-430 (tfhe_io.cu:1088-1137)
 *   export_/new_tfheGateBootstrappingSecretKeySet_*   tfhe_io.h:441-461 (tfhe_io.cu:1147-1201)
 *   export_/import_gate_bootstrapping_ciphertext_*    tfhe_io.h:473-499 (tfhe_io.cu:1214-1250)
 *   export_/import_lweSample_*                        tfhe_io.h:61-80   (tfhe_io.cu:90-139)
 *
 * File layout (all binary fields little-endian, as the reference writes them natively):
 *   text section   "-----BEGIN T-----\n" {"name: value\n" sorted by name} "-----END T-----\n"
 *                  longs "%ld", doubles "%.8lf"
 *   parameter set  GATEBOOTSPARAMS{ks_basebit,ks_t} LWEPARAMS{alpha_max,alpha_min,n}
 *                  TLWEPARAMS{N,alpha_max,alpha_min,k} TGSWPARAMS{Bgbit,l}
 *   cloud key      parameter set, LWEKSPARAMS{basebit,n,t},
 *                  i32 200, f64 max variance, KSK [N][t][base]{a[n], b}  (i32)
 *                  i32 201, f64 max variance, BK  [n][kpl][k+1][N]        (i32)
 *   secret key     cloud key, i32 43, lwe key [n], i32 169, tgsw key [k][N]
 *   ciphertext     i32 42, a[n], b, f64 current_variance
 *
 * Error behaviour follows the reference: a wrong type uid, a wrong section title or a
 * short read aborts (die_dramatically).  Parameter sets whose shape differs from the
 * default 128-bit set are rejected the same way (the MI355X engine is built for it).
 * Parameter sets, keysets and samples returned here are released with the tfhe.h
 * delete_* functions.
 */
#ifndef TFHE_AMD_TFHE_IO_H
#define TFHE_AMD_TFHE_IO_H

#include "tfhe_core.h"

#ifdef __cplusplus
#include <cstdio>
#include <iosfwd>
#else
#include <stdio.h>
#endif

EXPORT void export_lweSample_toFile(FILE *F, const LweSample *lwesample, const LweParams *params);
EXPORT void import_lweSample_fromFile(FILE *F, LweSample *lwesample, const LweParams *params);

EXPORT void export_tfheGateBootstrappingParameterSet_toFile(FILE *F, const TFheGateBootstrappingParameterSet *params);
EXPORT TFheGateBootstrappingParameterSet *new_tfheGateBootstrappingParameterSet_fromFile(FILE *F);

EXPORT void export_tfheGateBootstrappingCloudKeySet_toFile(FILE *F, const TFheGateBootstrappingCloudKeySet *params);
EXPORT TFheGateBootstrappingCloudKeySet *new_tfheGateBootstrappingCloudKeySet_fromFile(FILE *F);

EXPORT void export_tfheGateBootstrappingSecretKeySet_toFile(FILE *F, const TFheGateBootstrappingSecretKeySet *params);
EXPORT TFheGateBootstrappingSecretKeySet *new_tfheGateBootstrappingSecretKeySet_fromFile(FILE *F);

EXPORT void export_gate_bootstrapping_ciphertext_toFile(FILE *F, const LweSample *sample,
                                                        const TFheGateBootstrappingParameterSet *params);
EXPORT void import_gate_bootstrapping_ciphertext_fromFile(FILE *F, LweSample *sample,
                                                          const TFheGateBootstrappingParameterSet *params);

#ifdef __cplusplus
EXPORT void export_lweSample_toStream(std::ostream &F, const LweSample *lwesample, const LweParams *params);
EXPORT void import_lweSample_fromStream(std::istream &in, LweSample *lwesample, const LweParams *params);
EXPORT void export_tfheGateBootstrappingParameterSet_toStream(std::ostream &F,
                                                              const TFheGateBootstrappingParameterSet *params);
EXPORT TFheGateBootstrappingParameterSet *new_tfheGateBootstrappingParameterSet_fromStream(std::istream &F);
EXPORT void export_tfheGateBootstrappingCloudKeySet_toStream(std::ostream &F,
                                                             const TFheGateBootstrappingCloudKeySet *params);
EXPORT TFheGateBootstrappingCloudKeySet *new_tfheGateBootstrappingCloudKeySet_fromStream(std::istream &F);
EXPORT void export_tfheGateBootstrappingSecretKeySet_toStream(std::ostream &F,
                                                              const TFheGateBootstrappingSecretKeySet *params);
EXPORT TFheGateBootstrappingSecretKeySet *new_tfheGateBootstrappingSecretKeySet_fromStream(std::istream &F);
EXPORT void export_gate_bootstrapping_ciphertext_toStream(std::ostream &F, const LweSample *sample,
                                                          const TFheGateBootstrappingParameterSet *params);
EXPORT void import_gate_bootstrapping_ciphertext_fromStream(std::istream &F, LweSample *sample,
                                                            const TFheGateBootstrappingParameterSet *params);
#endif

#endif
