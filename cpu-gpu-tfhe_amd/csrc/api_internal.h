// api_internal.h — constructors shared by the Tier-1 API (tfhe_api.cpp) and the key /
// ciphertext file I/O (tfhe_io.cpp).  Not installed; the public surface is include/tfhe/.
#pragma once

#include <vector>

#include "params.h"
#include "../../include/tfhe/tfhe.h"

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
