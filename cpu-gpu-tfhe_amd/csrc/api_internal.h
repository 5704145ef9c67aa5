// api_internal.h — constructors shared by the Tier-1 API (tfhe_api.cpp) and the key /
// ciphertext file I/O (tfhe_io.cpp).  Not installed; the public surface is include/tfhe/.
#pragma once

#include <vector>

#include "params.h"
#include "../../include/tfhe/tfhe.h"
#include "../../include/tfhe_amd.h"

namespace tfhe_amd {
namespace api {

// One gate-bootstrapping parameter set and everything its pointers reach
// (tfhe_gate_bootstrapping.cu:25-55; tgsw.cu:7-29).  Only the default 128-bit shape is
// supported by the engine; the alphas are free because a set read back from a file holds
// the %.8lf-rounded values the writer printed.
struct ParamsImpl {
    LweParams in_out;
    TLweParams accum;
    Torus32 h[kL];
    TGswParams tgsw;
    TFheGateBootstrappingParameterSet set;
    explicit ParamsImpl(double lwe_alpha_min = kKsStdev, double lwe_alpha_max = kMaxStdev,
                        double tlwe_alpha_min = kBkStdev, double tlwe_alpha_max = kMaxStdev);
};

// registers p (owned by the registry from then on) and returns its public view
TFheGateBootstrappingParameterSet *register_params(ParamsImpl *p);
// dies when params was not made by this library
const ParamsImpl *params_of(const TFheGateBootstrappingParameterSet *params);

struct TGswKeyImpl {
    TGswKey pub;
    std::vector<int> coefs;   // k * N
    IntPolynomial poly;
};

LweKey *new_LweKey(const LweParams *params);
void delete_LweKey(LweKey *k);
TGswKey *new_tgsw_key(const ParamsImpl *P);                  // zero key
LweBootstrappingKey *new_bk(const ParamsImpl *P);            // zero BK + zero KSK
LweBootstrappingKeyFFT *new_bkfft(const LweBootstrappingKey *bk);

}  // namespace api
}  // namespace tfhe_amd

// tfhe_api.cpp <-> multi.cpp (multi-device batches)
// coefficient-domain bootstrapping key of a cloud key (int32 [500][4][2][1024])
int tfhe_amd_internal_bk_coef(const TFheGateBootstrappingCloudKeySet *bk, int32_t *out);
// one SoA batch of a gate on the key's Tier-1 device context (this thread's lane)
int tfhe_amd_internal_tier1_batch(const TFheGateBootstrappingCloudKeySet *bk, int gate, int B, int32_t *res_a,
                                  int32_t *res_b, const int32_t *a_a, const int32_t *a_b, const int32_t *b_a,
                                  const int32_t *b_b, const int32_t *c_a, const int32_t *c_b);
// compute units of a device (hipDeviceAttributeMultiprocessorCount, cached; 256 if unknown): the
// Tier-1 queue merges two batches while together they hold at most one ciphertext per CU
int tfhe_amd_internal_device_cus(int device);
// the extracted samples of a context's last gate batch (<= one round), halves x B rows of 1024
int tfhe_amd_internal_last_extracted(TfheAmdContext *c, int B, int halves, int32_t *u_a);
// device copy of host bytes on a context's GPU / its release; device-side current_variance of the
// context's last gate batch (engine.cpp)
int tfhe_amd_internal_upload(TfheAmdContext *c, const void *host, size_t bytes, void **dev);
void tfhe_amd_internal_free(int device, void *dev);
int tfhe_amd_internal_ks_variance(TfheAmdContext *c, int B, int halves, const double *d_var, double *out);
// the same for the context's last mixed-gate batch (gate i's variance in out[i])
int tfhe_amd_internal_mixed_variance(TfheAmdContext *c, int B, const double *d_var, double *out);
// Rows of an array of records that each point to their a[500] and hold b (and current_variance):
// record i is at base + i * stride; its a pointer at a_off, b at b_off, current_variance at v_off
// (tfhe_api.cpp: LweSample arrays, without the engine knowing the struct)
struct TfheAmdRows {
    char *base;
    size_t stride, a_off, b_off, v_off;
};
// a gate batch over such records (tfhe_amd_boots_batch): packed in parallel straight into the pinned
// staging buffer, pipelined in slices of one round (slice s + 1 packed and copied in while slice s
// computes, slice s - 1 unpacked meanwhile), current_variance of each result computed on the device
// from the KSK row variances d_var [1024][8][4] (k_ks_variance) and written with the result
int tfhe_amd_internal_gate_batch_rows(TfheAmdContext *c, int gate, int B, const TfheAmdRows *res,
                                      const TfheAmdRows *in, int nin, const double *d_var);
// drops the multi-device context registered for a key (tfhe_gpu_init) when the key is deleted
void tfhe_amd_internal_forget_multi(const void *bkfft);
// circuit.cpp: drops every circuit's device state (tables, scratch) held for a context; called by
// tfhe_amd_context_destroy (context uids are never reused, so a later context cannot inherit it)
void tfhe_amd_internal_circuits_forget_context(unsigned long long ctx_uid);
// the TFHE API's L1 entry points on host data (engine.cpp): op 0 = tGswFFTExternMulToTLwe (arg = key
// indices [B]), op 1 = tfhe_blindRotate_FFT (arg = bara [B][iters]); acc [B][2][1024] in place, exact
int tfhe_amd_internal_l1(TfheAmdContext *c, int op, int B, int iters, const int32_t *arg, int32_t *acc);
