// tfhe_api.cpp — the TFHE C API (Tier-1) over the MI355X engine.
//
// The drop-in boundary of SURVEY.md §8(b): the functions cpuParallel/Cipher.cpp and
// cloud.cpp call from libtfhe (bootsXXX, tfhe_bootstrap_(woKS_)FFT, lweKeySwitch, the
// key/ciphertext lifecycle and the LWE helpers).  Structs are allocated with the
// reference's layouts (include/tfhe/tfhe.h); the bootstrapped operations run on the GPU
// through a device context cached per key (engine.cpp).  Host-only pieces (key
// generation, encryption, linear LWE ops) restate the reference's CPU code and keep its
// RNG: std::default_random_engine seeded by tfhe_random_generator_setSeed
// (numeric-functions.cu:11-19), drawn in the reference's order.
//
// Reentrancy: every calling thread gets its own "lane" (stream + scratch) per key, so
// OpenMP callers (Cipher.cpp:116-120, cloud.cpp:390-393) run concurrently; the reference's
// global FFT scratch (lagrangehalfc_impl.cu:4) has no counterpart here.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <limits>
#include <map>
#include <memory>
#include <algorithm>
#include <mutex>
#include <random>
#include <unordered_map>
#include <vector>

#include "params.h"
#include "../../include/tfhe/tfhe.h"
#include "../../include/tfhe_amd.h"
#include "api_internal.h"

using namespace tfhe_amd;
using namespace tfhe_amd::api;

TfheAmdContext *tfhe_amd_context_lane(TfheAmdContext *primary);   // engine.cpp
int tfhe_amd_internal_unsliced_max();                                 // engine.cpp

// ------------------------------------------------------------------ numerics
// numeric-functions.cu:11-77

static std::default_random_engine generator;
static std::uniform_int_distribution<Torus32> uniformTorus32_distrib(INT32_MIN, INT32_MAX);
static std::mutex g_rng_mu;   // the reference RNG is global and not thread safe; we lock it

EXPORT void die_dramatically(const char *message) {
    std::cerr << message << std::endl;
    abort();
}

EXPORT void tfhe_random_generator_setSeed(uint32_t *values, int size) {
    std::lock_guard<std::mutex> lk(g_rng_mu);
    std::seed_seq seeds(values, values + size);
    generator.seed(seeds);
}

EXPORT Torus32 dtot32(double d) { return int32_t(int64_t((d - int64_t(d)) * 4294967296.0)); }
EXPORT double t32tod(Torus32 x) { return double(x) / 4294967296.0; }

static Torus32 gaussian32_nolock(Torus32 message, double sigma) {
    std::normal_distribution<double> distribution(0., sigma);   // fresh per draw, as :24
    double err = distribution(generator);
    return (Torus32)((uint32_t)message + (uint32_t)dtot32(err));
}
EXPORT Torus32 gaussian32(Torus32 message, double sigma) {
    std::lock_guard<std::mutex> lk(g_rng_mu);
    return gaussian32_nolock(message, sigma);
}

EXPORT Torus32 approxPhase(Torus32 phase, int Msize) {
    uint64_t interv = ((UINT64_C(1) << 63) / Msize) * 2;
    uint64_t half_interval = interv / 2;
    uint64_t phase64 = (uint64_t(uint32_t(phase)) << 32) + half_interval;
    phase64 -= phase64 % interv;
    return int32_t(phase64 >> 32);
}
EXPORT int modSwitchFromTorus32(Torus32 phase, int Msize) {
    uint64_t interv = ((UINT64_C(1) << 63) / Msize) * 2;
    uint64_t half_interval = interv / 2;
    uint64_t phase64 = (uint64_t(uint32_t(phase)) << 32) + half_interval;
    return int(phase64 / interv);
}
EXPORT Torus32 modSwitchToTorus32(int mu, int Msize) {
    uint64_t interv = ((UINT64_C(1) << 63) / Msize) * 2;
    uint64_t phase64 = uint64_t(int64_t(mu)) * interv;
    return Torus32(uint32_t(phase64 >> 32));
}

// ------------------------------------------------------------------ params
// tfhe_gate_bootstrapping.cu:25-55; tgsw.cu:7-29; tlwe.cu (extracted params n = k N)
// (ParamsImpl is declared in api_internal.h; alphas are arguments because parameter sets
// read back from a file carry the %.8lf-rounded values, tfhe_generic_streams.cu:37-41)

ParamsImpl::ParamsImpl(double lwe_alpha_min, double lwe_alpha_max, double tlwe_alpha_min, double tlwe_alpha_max)
    : in_out{kn, lwe_alpha_min, lwe_alpha_max},
      accum{kN, kK, tlwe_alpha_min, tlwe_alpha_max, LweParams{kN * kK, tlwe_alpha_min, tlwe_alpha_max}},
      tgsw{kL, kBgbit, 1 << kBgbit, (1 << kBgbit) / 2, (1u << kBgbit) - 1, &accum, kKpl, h, kDecompOffset},
      set{kKsT, kKsBasebit, &in_out, &tgsw} {
    for (int i = 0; i < kL; ++i) h[i] = Torus32(1u << (32 - (i + 1) * kBgbit));
}

static std::mutex g_params_mu;
static std::map<const TFheGateBootstrappingParameterSet *, ParamsImpl *> g_params;

TFheGateBootstrappingParameterSet *tfhe_amd::api::register_params(ParamsImpl *p) {
    std::lock_guard<std::mutex> lk(g_params_mu);
    g_params[&p->set] = p;
    return &p->set;
}

const ParamsImpl *tfhe_amd::api::params_of(const TFheGateBootstrappingParameterSet *params) {
    std::lock_guard<std::mutex> lk(g_params_mu);
    auto it = g_params.find(params);
    if (it == g_params.end()) die_dramatically("tfhe_amd: unknown parameter set");
    return it->second;
}

EXPORT TFheGateBootstrappingParameterSet *new_default_gate_bootstrapping_parameters(int minimum_lambda) {
    if (minimum_lambda > 128)
        die_dramatically("Sorry, for now, the parameters are only implemented for about 128bit of security!");
    return register_params(new ParamsImpl());
}

EXPORT void delete_gate_bootstrapping_parameters(TFheGateBootstrappingParameterSet *params) {
    std::lock_guard<std::mutex> lk(g_params_mu);
    auto it = g_params.find(params);
    if (it != g_params.end()) {
        delete it->second;
        g_params.erase(it);
    }
}

// ------------------------------------------------------------------ LWE samples
// lwesamples.cu, lwe-functions.cu:21-291

EXPORT LweSample *new_LweSample_array(int nbelts, const LweParams *params) {
    LweSample *s = (LweSample *)malloc(sizeof(LweSample) * (size_t)(nbelts > 0 ? nbelts : 1));
    for (int i = 0; i < nbelts; i++) {
        s[i].a = (Torus32 *)calloc((size_t)params->n, sizeof(Torus32));
        s[i].b = 0;
        s[i].current_variance = 0.;
    }
    return s;
}
EXPORT LweSample *new_LweSample(const LweParams *params) { return new_LweSample_array(1, params); }
EXPORT void delete_LweSample_array(int nbelts, LweSample *obj) {
    if (!obj) return;
    for (int i = 0; i < nbelts; i++) free(obj[i].a);
    free(obj);
}
EXPORT void delete_LweSample(LweSample *obj) { delete_LweSample_array(1, obj); }

EXPORT LweSample *new_gate_bootstrapping_ciphertext(const TFheGateBootstrappingParameterSet *params) {
    return new_LweSample(params->in_out_params);
}
EXPORT LweSample *new_gate_bootstrapping_ciphertext_array(int nbelems, const TFheGateBootstrappingParameterSet *params) {
    return new_LweSample_array(nbelems, params->in_out_params);
}
EXPORT void delete_gate_bootstrapping_ciphertext(LweSample *sample) { delete_LweSample(sample); }
EXPORT void delete_gate_bootstrapping_ciphertext_array(int nbelems, LweSample *samples) {
    delete_LweSample_array(nbelems, samples);
}

LweKey *tfhe_amd::api::new_LweKey(const LweParams *params) {
    LweKey *k = (LweKey *)malloc(sizeof(LweKey));
    *const_cast<const LweParams **>(&k->params) = params;
    k->key = (int *)calloc((size_t)params->n, sizeof(int));
    return k;
}
void tfhe_amd::api::delete_LweKey(LweKey *k) {
    if (!k) return;
    free(k->key);
    free(k);
}

static void lweKeyGen_nolock(LweKey *result) {
    std::uniform_int_distribution<int> distribution(0, 1);
    for (int i = 0; i < result->params->n; i++) result->key[i] = distribution(generator);
}
EXPORT void lweKeyGen(LweKey *result) {
    std::lock_guard<std::mutex> lk(g_rng_mu);
    lweKeyGen_nolock(result);
}

static void lweSymEncrypt_nolock(LweSample *result, Torus32 message, double alpha, const LweKey *key) {
    const int n = key->params->n;
    uint32_t b = (uint32_t)gaussian32_nolock(message, alpha);
    for (int i = 0; i < n; ++i) {
        result->a[i] = uniformTorus32_distrib(generator);
        b += (uint32_t)result->a[i] * (uint32_t)key->key[i];
    }
    result->b = (Torus32)b;
    result->current_variance = alpha * alpha;
}
EXPORT void lweSymEncrypt(LweSample *result, Torus32 message, double alpha, const LweKey *key) {
    std::lock_guard<std::mutex> lk(g_rng_mu);
    lweSymEncrypt_nolock(result, message, alpha, key);
}

static void lweSymEncryptWithExternalNoise_nolock(LweSample *result, Torus32 message, double noise, double alpha,
                                                  const LweKey *key) {
    const int n = key->params->n;
    uint32_t b = (uint32_t)message + (uint32_t)dtot32(noise);
    for (int i = 0; i < n; ++i) {
        result->a[i] = uniformTorus32_distrib(generator);
        b += (uint32_t)result->a[i] * (uint32_t)key->key[i];
    }
    result->b = (Torus32)b;
    result->current_variance = alpha * alpha;
}
EXPORT void lweSymEncryptWithExternalNoise(LweSample *result, Torus32 message, double noise, double alpha,
                                           const LweKey *key) {
    std::lock_guard<std::mutex> lk(g_rng_mu);
    lweSymEncryptWithExternalNoise_nolock(result, message, noise, alpha, key);
}

EXPORT Torus32 lwePhase(const LweSample *sample, const LweKey *key) {
    uint32_t axs = 0;
    for (int i = 0; i < key->params->n; ++i) axs += (uint32_t)sample->a[i] * (uint32_t)key->key[i];
    return (Torus32)((uint32_t)sample->b - axs);
}
EXPORT Torus32 lweSymDecrypt(const LweSample *sample, const LweKey *key, const int Msize) {
    return approxPhase(lwePhase(sample, key), Msize);
}

EXPORT void lweClear(LweSample *r, const LweParams *params) {
    for (int i = 0; i < params->n; ++i) r->a[i] = 0;
    r->b = 0;
    r->current_variance = 0.;
}
EXPORT void lweCopy(LweSample *r, const LweSample *s, const LweParams *params) {
    for (int i = 0; i < params->n; ++i) r->a[i] = s->a[i];
    r->b = s->b;
    r->current_variance = s->current_variance;
}
EXPORT void lweNegate(LweSample *r, const LweSample *s, const LweParams *params) {
    for (int i = 0; i < params->n; ++i) r->a[i] = (Torus32)(0u - (uint32_t)s->a[i]);
    r->b = (Torus32)(0u - (uint32_t)s->b);
    r->current_variance = s->current_variance;
}
EXPORT void lweNoiselessTrivial(LweSample *r, Torus32 mu, const LweParams *params) {
    for (int i = 0; i < params->n; ++i) r->a[i] = 0;
    r->b = mu;
    r->current_variance = 0.;
}
EXPORT void lweAddTo(LweSample *r, const LweSample *s, const LweParams *params) {
    for (int i = 0; i < params->n; ++i) r->a[i] = (Torus32)((uint32_t)r->a[i] + (uint32_t)s->a[i]);
    r->b = (Torus32)((uint32_t)r->b + (uint32_t)s->b);
    r->current_variance += s->current_variance;
}
EXPORT void lweSubTo(LweSample *r, const LweSample *s, const LweParams *params) {
    for (int i = 0; i < params->n; ++i) r->a[i] = (Torus32)((uint32_t)r->a[i] - (uint32_t)s->a[i]);
    r->b = (Torus32)((uint32_t)r->b - (uint32_t)s->b);
    r->current_variance += s->current_variance;
}
EXPORT void lweAddMulTo(LweSample *r, int p, const LweSample *s, const LweParams *params) {
    for (int i = 0; i < params->n; ++i) r->a[i] = (Torus32)((uint32_t)r->a[i] + (uint32_t)p * (uint32_t)s->a[i]);
    r->b = (Torus32)((uint32_t)r->b + (uint32_t)p * (uint32_t)s->b);
    r->current_variance += (p * p) * s->current_variance;
}
EXPORT void lweSubMulTo(LweSample *r, int p, const LweSample *s, const LweParams *params) {
    for (int i = 0; i < params->n; ++i) r->a[i] = (Torus32)((uint32_t)r->a[i] - (uint32_t)p * (uint32_t)s->a[i]);
    r->b = (Torus32)((uint32_t)r->b - (uint32_t)p * (uint32_t)s->b);
    r->current_variance += (p * p) * s->current_variance;
}

// ------------------------------------------------------------------ keys

// Private owners behind the public (reference-layout) structs.  The bootstrapping key is
// kept as one contiguous coefficient-domain block [kn][kpl][k+1][N] — the layout the device
// upload consumes — and the public TGswSample/TLweSample/TorusPolynomial views point into it.
struct BkImpl {
    LweBootstrappingKey pub;
    std::vector<int32_t> coef;                // [kn][4][2][kN]
    std::vector<TorusPolynomial> polys;       // kn*4*2 views
    std::vector<TLweSample> rows;             // kn*4
    std::vector<TLweSample *> blocs;          // kn*(k+1) bloc pointers
    std::vector<TGswSample> gsw;              // kn
    LweKeySwitchKey *ks;
};

struct KskImpl {
    LweKeySwitchKey pub;
    std::vector<int32_t> a;                   // [kN*8*4][kn]
    std::vector<LweSample> samples;           // kN*8*4
    std::vector<LweSample *> l1;              // kN*8
    std::vector<LweSample **> l0;             // kN
};

struct BkFFTImpl {
    LweBootstrappingKeyFFT pub;
    std::vector<int32_t> bk_coef;             // [kn][4][2][kN]   (NTT conversion happens on the GPU)
    LweKeySwitchKey *ks;                      // deep copy (owned)
    // pub.bkFFT: the reference's array of kn TGswSampleFFT (tgsw.h:78-96), so that callers can
    // pass bk->bkFFT + i to tGswFFTExternMulToTLwe; the samples themselves live on the GPU (null
    // all_samples) and an element maps back to (this key, i) through g_gsw (below)
    std::vector<TGswSampleFFT> gsw;
};

// key of every live TGswSampleFFT array: its first element -> the key (L1 entry points)
static std::mutex g_gsw_mu;
static std::map<const TGswSampleFFT *, BkFFTImpl *> g_gsw;
static BkFFTImpl *gsw_key_of(const TGswSampleFFT *p, int *index) {
    std::lock_guard<std::mutex> lk(g_gsw_mu);
    auto it = g_gsw.upper_bound(p);
    if (it == g_gsw.begin()) return nullptr;
    --it;
    const ptrdiff_t i = p - it->first;
    if (i < 0 || i >= (ptrdiff_t)it->second->gsw.size()) return nullptr;
    *index = (int)i;
    return it->second;
}

static KskImpl *ksk_of(const LweKeySwitchKey *k) { return reinterpret_cast<KskImpl *>(const_cast<LweKeySwitchKey *>(k)); }
static BkFFTImpl *bkfft_of(const LweBootstrappingKeyFFT *k) {
    return reinterpret_cast<BkFFTImpl *>(const_cast<LweBootstrappingKeyFFT *>(k));
}
static BkImpl *bk_of(const LweBootstrappingKey *k) { return reinterpret_cast<BkImpl *>(const_cast<LweBootstrappingKey *>(k)); }

static LweKeySwitchKey *new_ksk(const LweParams *out_params) {
    KskImpl *k = new KskImpl{LweKeySwitchKey{kN, kKsT, kKsBasebit, kKsBase, out_params, nullptr, nullptr, nullptr},
                             {}, {}, {}, {}};
    const size_t ns = (size_t)kN * kKsT * kKsBase;
    k->a.assign(ns * kn, 0);
    k->samples.resize(ns);
    for (size_t s = 0; s < ns; s++) k->samples[s] = LweSample{k->a.data() + s * kn, 0, 0.};
    k->l1.resize((size_t)kN * kKsT);
    for (size_t p = 0; p < k->l1.size(); p++) k->l1[p] = k->samples.data() + kKsBase * p;
    k->l0.resize(kN);
    for (int p = 0; p < kN; p++) k->l0[p] = k->l1.data() + kKsT * p;
    k->pub.ks0_raw = k->samples.data();
    k->pub.ks1_raw = k->l1.data();
    k->pub.ks = k->l0.data();
    return &k->pub;
}
static void delete_ksk(LweKeySwitchKey *k) { delete ksk_of(k); }

// flat [kN][8][4][kn+1] view of any LweKeySwitchKey (ours or foreign-built)
static void ksk_flatten(const LweKeySwitchKey *ks, int32_t *out) {
    for (int i = 0; i < kN; i++)
        for (int j = 0; j < kKsT; j++)
            for (int h = 0; h < kKsBase; h++) {
                const LweSample &s = ks->ks[i][j][h];
                int32_t *dst = out + (((size_t)i * kKsT + j) * kKsBase + h) * (kn + 1);
                memcpy(dst, s.a, sizeof(int32_t) * kn);
                dst[kn] = s.b;
            }
}

LweBootstrappingKey *tfhe_amd::api::new_bk(const ParamsImpl *P) {
    BkImpl *k = new BkImpl{LweBootstrappingKey{&P->in_out, &P->tgsw, &P->accum, &P->accum.extracted_lweparams,
                                               nullptr, nullptr},
                           {}, {}, {}, {}, {}, nullptr};
    k->coef.assign((size_t)kn * kKpl * 2 * kN, 0);
    k->polys.reserve((size_t)kn * kKpl * 2);
    for (size_t p = 0; p < (size_t)kn * kKpl * 2; p++) k->polys.push_back(TorusPolynomial{kN, k->coef.data() + p * kN});
    k->rows.reserve((size_t)kn * kKpl);
    for (size_t r = 0; r < (size_t)kn * kKpl; r++)
        k->rows.push_back(TLweSample{&k->polys[r * 2], &k->polys[r * 2 + 1], 0., kK});
    k->blocs.resize((size_t)kn * (kK + 1));
    for (int i = 0; i < kn; i++)
        for (int b = 0; b <= kK; b++) k->blocs[(size_t)i * (kK + 1) + b] = &k->rows[(size_t)i * kKpl + b * kL];
    k->gsw.reserve(kn);
    for (int i = 0; i < kn; i++)
        k->gsw.push_back(TGswSample{&k->rows[(size_t)i * kKpl], &k->blocs[(size_t)i * (kK + 1)], kK, kL});
    k->ks = new_ksk(&P->in_out);
    k->pub.bk = k->gsw.data();
    k->pub.ks = k->ks;
    return &k->pub;
}
static void delete_bk(LweBootstrappingKey *k) {
    if (!k) return;
    BkImpl *b = bk_of(k);
    delete_ksk(b->ks);
    delete b;
}

// coefficient BK of any LweBootstrappingKey -> flat [kn][4][2][kN]
static void bk_flatten(const LweBootstrappingKey *bk, int32_t *out) {
    for (int i = 0; i < kn; i++)
        for (int p = 0; p < kKpl; p++)
            for (int c = 0; c <= kK; c++)
                memcpy(out + (((size_t)i * kKpl + p) * 2 + c) * kN, bk->bk[i].all_sample[p].a[c].coefsT,
                       sizeof(int32_t) * kN);
}

// new_LweBootstrappingKeyFFT (lwe-bootstrapping-functions-fft.cu:2201 -> :60-89): copy the KSK,
// keep the coefficient BK for the device-side NTT conversion.
LweBootstrappingKeyFFT *tfhe_amd::api::new_bkfft(const LweBootstrappingKey *bk) {
    BkFFTImpl *f = new BkFFTImpl{LweBootstrappingKeyFFT{bk->in_out_params, bk->bk_params, bk->accum_params,
                                                        bk->extract_params, nullptr, nullptr},
                                 {}, nullptr};
    f->bk_coef.resize((size_t)kn * kKpl * 2 * kN);
    bk_flatten(bk, f->bk_coef.data());
    f->ks = new_ksk(bk->in_out_params);
    std::vector<int32_t> flat((size_t)kN * kKsT * kKsBase * (kn + 1));
    ksk_flatten(bk->ks, flat.data());
    KskImpl *dst = ksk_of(f->ks);
    for (size_t s = 0; s < dst->samples.size(); s++) {
        memcpy(dst->samples[s].a, flat.data() + s * (kn + 1), sizeof(int32_t) * kn);
        dst->samples[s].b = flat[s * (kn + 1) + kn];
        dst->samples[s].current_variance = bk->ks->ks0_raw[s].current_variance;
    }
    *const_cast<const LweKeySwitchKey **>(&f->pub.ks) = f->ks;
    f->gsw.reserve(kn);
    for (int i = 0; i < kn; ++i) f->gsw.push_back(TGswSampleFFT{nullptr, nullptr, kK, kL});
    *const_cast<const TGswSampleFFT **>(&f->pub.bkFFT) = f->gsw.data();
    std::lock_guard<std::mutex> lk(g_gsw_mu);
    g_gsw[f->gsw.data()] = f;
    return &f->pub;
}

static void forget_device_keys(const void *k1, const void *k2);

static void delete_bkfft(LweBootstrappingKeyFFT *k) {
    if (!k) return;
    BkFFTImpl *f = bkfft_of(k);
    {
        std::lock_guard<std::mutex> lk(g_gsw_mu);
        g_gsw.erase(f->gsw.data());
    }
    forget_device_keys(k, f->ks);
    tfhe_amd_internal_forget_multi(k);
    delete_ksk(f->ks);
    delete f;
}

TGswKey *tfhe_amd::api::new_tgsw_key(const ParamsImpl *P) {
    TGswKeyImpl *gk = new TGswKeyImpl{TGswKey{&P->tgsw, &P->accum, nullptr, TLweKey{&P->accum, nullptr}},
                                      std::vector<int>((size_t)kN * kK), IntPolynomial{kN, nullptr}};
    gk->poly.coefs = gk->coefs.data();
    gk->pub.key = &gk->poly;
    gk->pub.tlwe_key.key = &gk->poly;
    return &gk->pub;
}

// lweCreateKeySwitchKey (lwe-keyswitch-functions.cu:890-942)
static void create_ksk_nolock(LweKeySwitchKey *result, const int *in_key /*kN*/, const LweKey *out_key) {
    const int n = result->n, t = result->t, basebit = result->basebit, base = 1 << basebit;
    const double alpha = out_key->params->alpha_min;
    const int sizeks = n * t * (base - 1);
    std::vector<double> noise(sizeks);
    double err = 0;
    for (int i = 0; i < sizeks; ++i) {
        std::normal_distribution<double> distribution(0., alpha);
        noise[i] = distribution(generator);
        err += noise[i];
    }
    err = err / sizeks;
    for (int i = 0; i < sizeks; ++i) noise[i] -= err;
    int index = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < t; ++j) {
            lweNoiselessTrivial(&result->ks[i][j][0], 0, out_key->params);
            for (int h = 1; h < base; ++h) {
                Torus32 mess = (Torus32)((uint32_t)(in_key[i] * h) * (1u << (32 - (j + 1) * basebit)));
                lweSymEncryptWithExternalNoise_nolock(&result->ks[i][j][h], mess, noise[index], alpha, out_key);
                index += 1;
            }
        }
}

// tLweSymEncryptZero (tlwe-functions.cu:26-38) with an EXACT b += key * a (the reference
// uses its FFT multiply here, polynomials_arithmetic.h:112-114; key generation is
// client side and off the hot path)
static void tlwe_encrypt_zero_nolock(TLweSample *r, double alpha, const int *key /*kN binary*/) {
    uint32_t *b = (uint32_t *)r->b->coefsT;
    for (int j = 0; j < kN; ++j) b[j] = (uint32_t)gaussian32_nolock(0, alpha);
    uint32_t *a = (uint32_t *)r->a[0].coefsT;
    for (int j = 0; j < kN; ++j) a[j] = (uint32_t)uniformTorus32_distrib(generator);   // torusPolynomialUniform
    for (int s = 0; s < kN; ++s) {
        if (!key[s]) continue;           // b += X^s * a (negacyclic)
        for (int i = 0; i < s; ++i) b[i] -= a[i - s + kN];
        for (int i = s; i < kN; ++i) b[i] += a[i - s];
    }
    r->current_variance = alpha * alpha;
}

EXPORT TFheGateBootstrappingSecretKeySet *
new_random_gate_bootstrapping_secret_keyset(const TFheGateBootstrappingParameterSet *params) {
    const ParamsImpl *P = params_of(params);
    std::lock_guard<std::mutex> lk(g_rng_mu);
    LweKey *lwe_key = new_LweKey(params->in_out_params);
    lweKeyGen_nolock(lwe_key);                                              // :60
    TGswKeyImpl *gk = reinterpret_cast<TGswKeyImpl *>(new_tgsw_key(P));
    {   // tGswKeyGen -> tLweKeyGen (tlwe-functions.cu:15-23)
        std::uniform_int_distribution<int> distribution(0, 1);
        for (int j = 0; j < kN; ++j) gk->coefs[j] = distribution(generator);
    }
    // tfhe_createLweBootstrappingKey (lwe-bootstrapping-functions.cu:185-217)
    LweBootstrappingKey *bk = new_bk(P);
    create_ksk_nolock(bk->ks, gk->coefs.data(), lwe_key);   // extracted key = tlwe key coefs (k = 1)
    const double alpha = P->accum.alpha_min;
    for (int i = 0; i < kn; i++) {
        TGswSample *g = &bk->bk[i];
        for (int p = 0; p < kKpl; ++p) tlwe_encrypt_zero_nolock(&g->all_sample[p], alpha, gk->coefs.data());
        // tGswAddMuIntH (tgsw-functions.cu:114-124)
        for (int bloc = 0; bloc <= kK; ++bloc)
            for (int l = 0; l < kL; l++) {
                Torus32 *c0 = &g->bloc_sample[bloc][l].a[bloc].coefsT[0];
                *c0 = (Torus32)((uint32_t)*c0 + (uint32_t)lwe_key->key[i] * (uint32_t)P->h[l]);
            }
    }
    LweBootstrappingKeyFFT *bkfft = new_bkfft(bk);
    return new TFheGateBootstrappingSecretKeySet{params, lwe_key, &gk->pub,
                                                 TFheGateBootstrappingCloudKeySet{params, bk, bkfft}};
}

EXPORT void delete_gate_bootstrapping_secret_keyset(TFheGateBootstrappingSecretKeySet *keyset) {
    if (!keyset) return;
    delete_bkfft(const_cast<LweBootstrappingKeyFFT *>(keyset->cloud.bkFFT));
    delete_bk(const_cast<LweBootstrappingKey *>(keyset->cloud.bk));
    delete reinterpret_cast<TGswKeyImpl *>(const_cast<TGswKey *>(keyset->tgsw_key));
    delete_LweKey(const_cast<LweKey *>(keyset->lwe_key));
    delete keyset;
}

EXPORT void delete_gate_bootstrapping_cloud_keyset(TFheGateBootstrappingCloudKeySet *keyset) {
    if (!keyset) return;
    delete_bkfft(const_cast<LweBootstrappingKeyFFT *>(keyset->bkFFT));
    delete_bk(const_cast<LweBootstrappingKey *>(keyset->bk));
    delete keyset;
}

EXPORT void bootsSymEncrypt(LweSample *result, int message, const TFheGateBootstrappingSecretKeySet *key) {
    Torus32 _1s8 = modSwitchToTorus32(1, 8);
    Torus32 mu = message ? _1s8 : -_1s8;
    double alpha = key->params->in_out_params->alpha_min;
    lweSymEncrypt(result, mu, alpha, key->lwe_key);
}
EXPORT int bootsSymDecrypt(const LweSample *sample, const TFheGateBootstrappingSecretKeySet *key) {
    Torus32 mu = lwePhase(sample, key->lwe_key);
    return mu > 0 ? 1 : 0;
}

// ------------------------------------------------------------------ device contexts

static std::atomic<int> g_default_device{0};

// One pending single-gate call of the coalescing queue (below).
// Its caller sleeps on the request's own condition variable, so that a finished batch wakes only
// its own callers (and a freed lane one new leader) instead of every thread inside a call.
struct Tier1Req {
    int gate;
    LweSample *r;
    const LweSample *a, *b, *c;
    bool taken = false;   // in a running batch (queue lock)

    int rc = TFHE_AMD_OK;
    std::mutex m;             // wake-up of the caller: done (its batch finished) or a call to lead
    std::condition_variable cv;
    bool signaled = false, done = false;
    // a finished batch's callers are woken as a binary tree over wl: the leader wakes wl[0], wl[1],
    // and the caller at wl[i] wakes wl[2i + 2], wl[2i + 3] (log2 depth instead of one by one)
    std::shared_ptr<std::vector<Tier1Req *>> wl;
    int wi = -1;
    void wake(bool finished) {   // the request may be gone once m is released with done set
        std::lock_guard<std::mutex> lk(m);
        done = done || finished;
        signaled = true;
        cv.notify_one();
    }
};

// Coalescing queue of the Tier-1 gates of one key ("per-thread streams or a
// batching queue").  The reference's CPU callers enter single gates from OpenMP teams
// (Cipher.cpp:83-120, cloud.cpp:389-395); one B = 1 launch per call would occupy 2 waves of one
// CU each, and a process has only 4 hardware queues.  Here a call enqueues its gate; a waiting
// thread becomes the leader of the next batch when a queue lane is free and no other leader is
// collecting: it waits until every thread inside a gate call and not already in a running batch
// has enqueued (at most the adaptive window below), takes every pending gate and runs them on
// that lane — one gate kind as a gate batch, several kinds as one mixed launch per 512 gates.
// Two lanes (own stream + scratch each) alternate, so batch k + 1 is staged and launched while
// batch k is still on the GPU or being unstaged: the queue no longer serialises a whole batch's
// host work with the next one — once the two together exceed one ciphertext per CU; below that
// the next leader waits for the running batch and merges its callers' next gates into one launch.  A lone thread is its own leader at once (B = 1 latency).  Callers
// sleep on their own request: a finished batch's leader does its callers' bookkeeping and wakes
// exactly them, and a freed lane wakes the oldest pending caller to lead (no wake-up of every
// thread in the call per batch, which serialised 64 threads on the queue lock).
// The window adapts to the callers: it starts at the floor below (200 us),
// follows 4x the average wait that ended with every expected thread enqueued (+ 20 us), and
// shrinks by a quarter after a wait that timed out (callers busy elsewhere), within [200, 1000] us.
constexpr int kQueueLanes = 2;
// the straggler window never drops below this: released callers come back within ~0.1 ms, and a
// window that times out on them splits a team into partial batches (which then queue behind each
// other); a caller that does not come back costs one such wait, after which it is no longer expected
constexpr double kWindowFloorUs = 200.0;
struct Coalescer {
    std::mutex mu;
    std::condition_variable arrive_cv;   // a collecting leader waits here for stragglers
    std::vector<Tier1Req *> pending;
    int inside = 0;       // threads inside a Tier-1 gate call on this key
    int in_flight = 0;    // gates taken by running batches
    int running = 0;      // batches running (<= kQueueLanes)
    int returning = 0;    // callers released by finished batches, expected back with their next gate
    bool collecting = false;   // a leader is waiting for stragglers
    bool lane_busy[kQueueLanes] = {false, false};
    int merge_limit = 256;     // gates two lanes' batches may hold together and still merge: one
                               // ciphertext per CU of the key's device (set when the key registers)
    double window_us = -1.0;   // adaptive straggler window (set on first use)
    double wait_avg_us = 0.0;
    long long batches = 0, gates = 0, largest = 0, overlapped = 0;
    // where a batch's time goes (ms, summed over batches; tfhe_amd_tier1_queue_times):
    // 0 the leader's straggler wait, 1 packing, 2 the device gate batch (staging, copies, kernels,
    // synchronize), 3 the current_variance sums on the device (mixed kinds; single-kind batches
    // sum them inside 2), 4 unpacking
    double ms[5] = {0, 0, 0, 0, 0};
};

struct KeyEntry {
    uint64_t id;
    const LweKeySwitchKey *ks = nullptr;
    TfheAmdContext *primary = nullptr;
    std::vector<TfheAmdContext *> lanes;
    std::mutex mu;
    Coalescer q;
    TfheAmdContext *qlane[kQueueLanes] = {nullptr, nullptr};   // the queue's lanes (one leader each at a time)
    double *d_var = nullptr;           // KSK row variances [1024][8][4] on the primary's device
};
static std::mutex g_reg_mu;
static std::unordered_map<const void *, std::shared_ptr<KeyEntry>> g_reg;   // bkFFT or KSK -> entry
static std::atomic<uint64_t> g_next_id{1};

static std::shared_ptr<KeyEntry> entry_for(const LweBootstrappingKeyFFT *bkfft, const LweKeySwitchKey *ks) {
    const void *k = bkfft ? (const void *)bkfft : (const void *)ks;
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.find(k);
    if (it != g_reg.end()) return it->second;
    if (!bkfft) {   // a KSK that belongs to a registered bkFFT shares its context
        for (auto &kv : g_reg)
            if (kv.second->ks == ks) return kv.second;
    }
    std::vector<int32_t> flat_ks((size_t)kN * kKsT * kKsBase * (kn + 1));
    const int32_t *bk_coef = nullptr;
    if (bkfft) {
        bk_coef = bkfft_of(bkfft)->bk_coef.data();
        ksk_flatten(bkfft->ks, flat_ks.data());
    } else {
        ksk_flatten(ks, flat_ks.data());
    }
    auto e = std::make_shared<KeyEntry>();
    e->id = g_next_id++;
    e->ks = bkfft ? bkfft->ks : ks;
    int rc = tfhe_amd_context_create_raw(bk_coef, flat_ks.data(), g_default_device.load(), &e->primary);
    if (rc != TFHE_AMD_OK) {
        fprintf(stderr, "tfhe_amd: cannot create the device context (rc=%d): no usable MI355X/HIP device\n", rc);
        die_dramatically("tfhe_amd: GPU engine unavailable");
    }
    e->q.merge_limit = tfhe_amd_internal_device_cus(tfhe_amd_context_device(e->primary));
    g_reg[k] = e;
    return e;
}

static void forget_device_keys(const void *k1, const void *k2) {
    std::vector<std::shared_ptr<KeyEntry>> dead;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        for (const void *k : {k1, k2}) {
            auto it = g_reg.find(k);
            if (it != g_reg.end()) {
                dead.push_back(it->second);
                g_reg.erase(it);
            }
        }
    }
    for (auto &e : dead) {
        std::lock_guard<std::mutex> lk(e->mu);
        for (auto *l : e->lanes) tfhe_amd_context_destroy(l);
        e->lanes.clear();
        for (auto *&ql : e->qlane) {
            if (ql) tfhe_amd_context_destroy(ql);
            ql = nullptr;
        }
        if (e->d_var) tfhe_amd_internal_free(tfhe_amd_context_device(e->primary), e->d_var);
        e->d_var = nullptr;
        tfhe_amd_context_destroy(e->primary);
        e->primary = nullptr;
    }
}

// This thread's lanes (own stream + scratch) on each key's device.  A thread that exits gives
// its lanes back (the holder's destructor), so callers that spawn short-lived threads (a
// std::thread per request, non-pooled OpenMP teams) do not accumulate streams, scratch and
// pinned memory per thread; a key deleted first has already destroyed its lanes (the weak
// reference is then expired, or the lane is no longer listed).
struct LaneHolder {
    struct Slot {
        std::weak_ptr<KeyEntry> entry;
        TfheAmdContext *lane;
    };
    std::unordered_map<uint64_t, Slot> slots;
    ~LaneHolder() {
        for (auto &kv : slots) {
            std::shared_ptr<KeyEntry> e = kv.second.entry.lock();
            if (!e) continue;
            std::lock_guard<std::mutex> lk(e->mu);
            auto it = std::find(e->lanes.begin(), e->lanes.end(), kv.second.lane);
            if (it == e->lanes.end()) continue;
            e->lanes.erase(it);
            tfhe_amd_context_destroy(kv.second.lane);
        }
    }
};

static TfheAmdContext *lane_for(const LweBootstrappingKeyFFT *bkfft, const LweKeySwitchKey *ks) {
    thread_local LaneHolder holder;
    std::shared_ptr<KeyEntry> e = entry_for(bkfft, ks);
    auto it = holder.slots.find(e->id);
    if (it != holder.slots.end()) return it->second.lane;
    std::lock_guard<std::mutex> lk(e->mu);
    TfheAmdContext *l = tfhe_amd_context_lane(e->primary);
    if (!l) die_dramatically("tfhe_amd: cannot create a per-thread GPU lane");
    e->lanes.push_back(l);
    holder.slots[e->id] = LaneHolder::Slot{e, l};
    return l;
}

// lanes currently alive for the Tier-1 key of `bk` (tests: threads give their lanes back)
EXPORT int tfhe_amd_tier1_lane_count(const TFheGateBootstrappingCloudKeySet *bk) {
    if (!bk || !bk->bkFFT) return TFHE_AMD_E_ARG;
    std::shared_ptr<KeyEntry> e;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_reg.find(bk->bkFFT);
        if (it == g_reg.end()) return 0;
        e = it->second;
    }
    std::lock_guard<std::mutex> lk(e->mu);
    return (int)e->lanes.size();
}

EXPORT int tfhe_amd_set_default_device(int device) {
    if (device < 0) return TFHE_AMD_E_ARG;
    g_default_device = device;
    return TFHE_AMD_OK;
}

EXPORT int tfhe_amd_context_create(const TFheGateBootstrappingCloudKeySet *bk, int device, TfheAmdContext **out) {
    if (!bk || !bk->bkFFT || !out) return TFHE_AMD_E_ARG;
    std::vector<int32_t> flat_ks((size_t)kN * kKsT * kKsBase * (kn + 1));
    ksk_flatten(bk->bkFFT->ks, flat_ks.data());
    return tfhe_amd_context_create_raw(bkfft_of(bk->bkFFT)->bk_coef.data(), flat_ks.data(), device, out);
}

EXPORT int tfhe_amd_export_bk(const TFheGateBootstrappingCloudKeySet *bk, int32_t *out) {
    if (!bk || !bk->bk || !out) return TFHE_AMD_E_ARG;
    bk_flatten(bk->bk, out);
    return TFHE_AMD_OK;
}
EXPORT int tfhe_amd_export_ksk(const TFheGateBootstrappingCloudKeySet *bk, int32_t *out) {
    if (!bk || !bk->bkFFT || !out) return TFHE_AMD_E_ARG;
    ksk_flatten(bk->bkFFT->ks, out);
    return TFHE_AMD_OK;
}
EXPORT int tfhe_amd_export_lwe_key(const TFheGateBootstrappingSecretKeySet *key, int32_t *out) {
    if (!key || !out) return TFHE_AMD_E_ARG;
    memcpy(out, key->lwe_key->key, sizeof(int32_t) * kn);
    return TFHE_AMD_OK;
}

EXPORT int tfhe_amd_export_tlwe_key(const TFheGateBootstrappingSecretKeySet *key, int32_t *out) {
    if (!key || !out) return TFHE_AMD_E_ARG;
    memcpy(out, key->tgsw_key->tlwe_key.key[0].coefs, sizeof(int32_t) * kN);
    return TFHE_AMD_OK;
}

// ------------------------------------------------------------------ bootstrapping API

static void check(int rc, const char *what) {
    if (rc != TFHE_AMD_OK) {
        fprintf(stderr, "tfhe_amd: %s failed (rc=%d)\n", what, rc);
        die_dramatically("tfhe_amd: GPU engine error");
    }
}

// current_variance of a key-switched sample, as the reference computes it: lweKeySwitch
// (lwe-keyswitch-functions.cu:955-987) starts from lweNoiselessTrivial (variance 0) and every
// lweSubTo of a key-switching-key row (lweKeySwitchTranslate_fromArray :101-127) adds that row's
// variance (lwe-functions.cu:150), in the same i, j order (so the double sum is the same).
// Bookkeeping only: excluded from the Torus32 parity.
static double ks_variance(const LweKeySwitchKey *ks, const int32_t *u_a) {
    const uint32_t prec = 1u << (32 - (1 + ks->basebit * ks->t));
    const uint32_t mask = (uint32_t)ks->base - 1;
    double v = 0.;
    for (int i = 0; i < ks->n; ++i) {
        const uint32_t aibar = (uint32_t)u_a[i] + prec;
        for (int j = 0; j < ks->t; ++j) {
            const uint32_t aij = (aibar >> (32 - (j + 1) * ks->basebit)) & mask;
            if (aij) v += ks->ks[i][j][aij].current_variance;
        }
    }
    return v;
}

// the key-switch input of a lane's last gate batch (one sample, halves = 2 for MUX: u1 + u2)
static void ks_input_of_last(TfheAmdContext *l, int B, int halves, std::vector<int32_t> &u) {
    u.resize((size_t)halves * B * kN);
    check(tfhe_amd_internal_last_extracted(l, B, halves, u.data()), "variance bookkeeping");
    if (halves == 2)
        for (size_t j = 0; j < (size_t)B * kN; ++j)
            u[j] = (int32_t)((uint32_t)u[j] + (uint32_t)u[(size_t)B * kN + j]);
}

EXPORT void tfhe_bootstrap_woKS_FFT(LweSample *result, const LweBootstrappingKeyFFT *bk, Torus32 mu,
                                    const LweSample *x) {
    TfheAmdContext *l = lane_for(bk, nullptr);
    check(tfhe_amd_bootstrap_woks_batch_host(l, 1, mu, x->a, &x->b, result->a, &result->b), "tfhe_bootstrap_woKS_FFT");
    // the reference's extraction (lwe.cu:41-56, 227-237) leaves current_variance as it was
}

EXPORT void tfhe_bootstrap_FFT(LweSample *result, const LweBootstrappingKeyFFT *bk, Torus32 mu, const LweSample *x) {
    TfheAmdContext *l = lane_for(bk, nullptr);
    check(tfhe_amd_bootstrap_batch_host(l, 1, mu, x->a, &x->b, result->a, &result->b), "tfhe_bootstrap_FFT");
    std::vector<int32_t> u;
    ks_input_of_last(l, 1, 1, u);
    result->current_variance = ks_variance(bk->ks, u.data());
}

EXPORT void lweKeySwitch(LweSample *result, const LweKeySwitchKey *ks, const LweSample *sample) {
    TfheAmdContext *l = lane_for(nullptr, ks);
    const double v = ks_variance(ks, sample->a);   // before: result may alias sample
    check(tfhe_amd_keyswitch_batch_host(l, 1, sample->a, &sample->b, result->a, &result->b), "lweKeySwitch");
    result->current_variance = v;
}

// ------------------------------------------------------------------ L1: blind rotation parts
// tfhe.h:42-43 (lwe-bootstrapping-functions-fft.cu:676-737, 1408-1456) and tgsw_functions.h:70
// (tgsw-fft-operations.cu:124-264) on the key's GPU context, exact (the NTT kernel's arithmetic):
// a caller that holds bk->bkFFT->bkFFT can drive the loop itself, as the reference allows.

struct TorusPolyImpl {
    TorusPolynomial pub;
    std::vector<Torus32> c;
};
struct TLweSampleImpl {
    TLweSample pub;
    std::vector<Torus32> coefs;
    std::vector<TorusPolynomial> polys;
};
// tlwe.h:222, polynomials.h:97 (allocation + construction; coefficients zero)
EXPORT TorusPolynomial *new_TorusPolynomial(const int N) {
    if (N <= 0) die_dramatically("new_TorusPolynomial: N must be positive");
    TorusPolyImpl *p = new TorusPolyImpl{TorusPolynomial{N, nullptr}, std::vector<Torus32>((size_t)N, 0)};
    p->pub.coefsT = p->c.data();
    return &p->pub;
}
EXPORT void delete_TorusPolynomial(TorusPolynomial *obj) { delete reinterpret_cast<TorusPolyImpl *>(obj); }
EXPORT TLweSample *new_TLweSample(const TLweParams *params) {
    const int k = params->k, N = params->N;
    TLweSampleImpl *t = new TLweSampleImpl{TLweSample{nullptr, nullptr, 0., k}, std::vector<Torus32>((size_t)(k + 1) * N, 0), {}};
    t->polys.reserve(k + 1);
    for (int i = 0; i <= k; ++i) t->polys.push_back(TorusPolynomial{N, t->coefs.data() + (size_t)i * N});
    t->pub.a = t->polys.data();
    t->pub.b = t->pub.a + k;
    return &t->pub;
}
EXPORT void delete_TLweSample(TLweSample *obj) { delete reinterpret_cast<TLweSampleImpl *>(obj); }

static BkFFTImpl *l1_key(const TGswSampleFFT *gsw, const TGswParams *params, int *index) {
    BkFFTImpl *f = gsw ? gsw_key_of(gsw, index) : nullptr;
    if (!f) die_dramatically("tfhe_amd: TGswSampleFFT pointer is not part of a bootstrapping key of this library");
    if (params && (params->tlwe_params->N != kN || params->tlwe_params->k != kK || params->l != kL))
        die_dramatically("tfhe_amd: only the default gate-bootstrapping parameter set is supported");
    return f;
}
static void tlwe_to_flat(const TLweSample *s, int32_t *acc) {
    memcpy(acc, s->a[0].coefsT, sizeof(int32_t) * kN);
    memcpy(acc + kN, s->b->coefsT, sizeof(int32_t) * kN);
}
static void flat_to_tlwe(const int32_t *acc, TLweSample *s) {
    memcpy(s->a[0].coefsT, acc, sizeof(int32_t) * kN);
    memcpy(s->b->coefsT, acc + kN, sizeof(int32_t) * kN);
}

// accum <- gsw (x) accum; current_variance 0 as the reference's tLweFFTClear leaves it
EXPORT void tGswFFTExternMulToTLwe(TLweSample *accum, const TGswSampleFFT *gsw, const TGswParams *params) {
    int i = 0;
    BkFFTImpl *f = l1_key(gsw, params, &i);
    std::vector<int32_t> acc(2 * kN);
    tlwe_to_flat(accum, acc.data());
    check(tfhe_amd_internal_l1(lane_for(&f->pub, nullptr), 0, 1, 0, &i, acc.data()), "tGswFFTExternMulToTLwe");
    flat_to_tlwe(acc.data(), accum);
    accum->current_variance = 0.;
}

// n CMux steps with keys bk[0..n) (bk = an element of a key's array; bara_i == 0 skipped, :705);
// current_variance unchanged (each tfhe_MuxRotate_FFT adds the accumulator's to a zero one)
EXPORT void tfhe_blindRotate_FFT(TLweSample *accum, const TGswSampleFFT *bk, const int *bara, const int n,
                                 const TGswParams *bk_params) {
    int i0 = 0;
    BkFFTImpl *f = l1_key(bk, bk_params, &i0);
    if (n < 0 || i0 + n > kn) die_dramatically("tfhe_blindRotate_FFT: n keys past the end of the key");
    if (n == 0) return;
    std::vector<int32_t> acc(2 * kN), a(kn, 0);
    tlwe_to_flat(accum, acc.data());
    // keys i0 .. i0 + n - 1: steps before i0 are identity (a = 0)
    for (int i = 0; i < n; ++i) a[i0 + i] = (int32_t)(((bara[i] % k2N) + k2N) % k2N);
    check(tfhe_amd_internal_l1(lane_for(&f->pub, nullptr), 1, 1, i0 + n, a.data(), acc.data()),
          "tfhe_blindRotate_FFT");
    flat_to_tlwe(acc.data(), accum);
}

// ACC = (0, X^{2N - barb} v) (v itself for barb = 0), blind rotation, extraction at index 0
// (lwe.cu:41-56): result has dimension N; its current_variance is left as it was (lwe.cu)
EXPORT void tfhe_blindRotateAndExtract_FFT(LweSample *result, const TorusPolynomial *v, const TGswSampleFFT *bk,
                                           const int barb, const int *bara, const int n,
                                           const TGswParams *bk_params) {
    int i0 = 0;
    BkFFTImpl *f = l1_key(bk, bk_params, &i0);
    if (n < 0 || i0 + n > kn) die_dramatically("tfhe_blindRotateAndExtract_FFT: n keys past the end of the key");
    std::vector<int32_t> acc(2 * kN, 0), a(kn, 0);
    const int e = ((k2N - barb) % k2N + k2N) % k2N;   // torusPolynomialMulByXai(2N - barb)
    for (int j = 0; j < kN; ++j) {                   // acc_b[j] = (X^e v)[j]
        int src = j - e;
        uint32_t sign = 0;
        while (src < 0) { src += kN; sign ^= 1; }
        const uint32_t x = (uint32_t)v->coefsT[src];
        acc[kN + j] = (int32_t)(sign ? 0u - x : x);
    }
    if (n > 0) {
        for (int i = 0; i < n; ++i) a[i0 + i] = (int32_t)(((bara[i] % k2N) + k2N) % k2N);
        check(tfhe_amd_internal_l1(lane_for(&f->pub, nullptr), 1, 1, i0 + n, a.data(), acc.data()),
              "tfhe_blindRotateAndExtract_FFT");
    }
    result->a[0] = acc[0];
    for (int j = 1; j < kN; ++j) result->a[j] = (int32_t)(0u - (uint32_t)acc[kN - j]);
    result->b = acc[kN];
}

// ------------------------------------------------------------------ gates

// TFHE_AMD_TIER1_COALESCE=0: every thread runs its own B = 1 batches on its own lane (no queue)
static bool coalesce_enabled() {
    static const bool on = [] {
        const char *e = getenv("TFHE_AMD_TIER1_COALESCE");
        return !(e && e[0] == '0');
    }();
    return on;
}

static double *ks_variance_table(const TFheGateBootstrappingCloudKeySet *bk) {
    // the KSK row variances on the device, once per key: each slice's current_variance is summed by
    // k_ks_variance (the reference's order of double adds) instead of on the host from the slice's
    // 4 KB-per-gate key-switch inputs (B = 1024: ~16 ms of host work and a 4 MB copy)
    std::shared_ptr<KeyEntry> e = entry_for(bk->bkFFT, nullptr);
    std::lock_guard<std::mutex> lk(e->mu);
    if (!e->d_var) {
        const LweKeySwitchKey *ks = bk->bkFFT->ks;
        std::vector<double> var(kKsVarWords, 0.0);
        bool uniform = true;
        const double v0 = ks->ks[0][0][1].current_variance;
        for (int i = 0; i < kN; ++i)
            for (int j = 0; j < kKsT; ++j)
                for (int h = 0; h < kKsBase; ++h) {
                    const double v = ks->ks[i][j][h].current_variance;
                    var[((size_t)i * kKsT + j) * kKsBase + h] = v;
                    if (h && memcmp(&v, &v0, sizeof v) != 0) uniform = false;   // rows a digit selects
                }
        if (uniform) {   // the sums of k equal terms, added one at a time as the reference does
            var[kKsVarUniform] = 1.0;
            double acc = 0.0;
            for (int k = 0; k <= kN * kKsT; ++k) {
                var[kKsVarUniform + 1 + k] = acc;
                acc += v0;
            }
        }
        void *dv = nullptr;
        if (tfhe_amd_internal_upload(e->primary, var.data(), sizeof(double) * var.size(), &dv)) return nullptr;
        e->d_var = (double *)dv;
    }
    return e->d_var;
}

// A batch of queued gates holding more than one gate kind runs as ONE mixed launch per 512 gates
// (tfhe_amd_gate_batch_mixed_host: one blind rotation + one key switch for all kinds; run_tier1_batch
// below takes the single-kind batches).  Inputs are staged before anything is written, so a result
// may alias any input of its own call; current_variance comes from the device
// (tfhe_amd_internal_mixed_variance, in the reference's order of adds).
using Tier1Clock = std::chrono::steady_clock;
static double ms_since(Tier1Clock::time_point &t) {
    const Tier1Clock::time_point now = Tier1Clock::now();
    const double d = std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
    return d;
}

static void run_tier1_mixed(TfheAmdContext *l, const std::vector<Tier1Req *> &batch, double *ms,
                            const double *d_var) {
    Tier1Clock::time_point t = Tier1Clock::now();
    std::vector<int32_t> buf;
    std::vector<int> gates;
    std::vector<double> var;
    const int total = (int)batch.size();
    for (int s0 = 0; s0 < total; s0 += 512) {
        const int n = std::min(512, total - s0);
        const size_t A = (size_t)n * kn;
        buf.resize(4 * A + 4 * (size_t)n);   // every word the launch reads is written below
        int32_t *aa = buf.data(), *ba = aa + A, *ca = ba + A, *ra = ca + A;
        int32_t *ab = ra + A, *bb = ab + n, *cb = bb + n, *rb = cb + n;
        gates.resize(n);
        for (int i = 0; i < n; ++i) {
            const Tier1Req *q = batch[s0 + i];
            gates[i] = q->gate;
            memcpy(aa + (size_t)i * kn, q->a->a, kn * 4); ab[i] = q->a->b;
            memcpy(ba + (size_t)i * kn, q->b->a, kn * 4); bb[i] = q->b->b;
            if (q->gate == TFHE_GATE_MUX) { memcpy(ca + (size_t)i * kn, q->c->a, kn * 4); cb[i] = q->c->b; }
        }
        ms[1] += ms_since(t);
        int rc = tfhe_amd_gate_batch_mixed_host(l, n, gates.data(), ra, rb, aa, ab, ba, bb, ca, cb);
        ms[2] += ms_since(t);
        // current_variance on the device from the launch's own key-switch table (a MUX's u1 + u2)
        var.resize(n);
        if (rc == TFHE_AMD_OK) rc = tfhe_amd_internal_mixed_variance(l, n, d_var, var.data());
        ms[3] += ms_since(t);
        if (rc != TFHE_AMD_OK) {
            for (int i = s0; i < total; ++i) batch[i]->rc = rc;
            return;
        }
        for (int i = 0; i < n; ++i) {
            Tier1Req *q = batch[s0 + i];
            memcpy(q->r->a, ra + (size_t)i * kn, kn * 4);
            q->r->b = rb[i];
            q->r->current_variance = var[i];
        }
        ms[4] += ms_since(t);
    }
}

// One gate kind: the engine's record path (tfhe_amd_internal_gate_batch_rows) gathers each request's
// input rows straight into the lane's pinned staging, scatters the results straight into the callers'
// result samples and sums current_variance on the device, so the batch has no intermediate SoA copies,
// no readback of the key-switch inputs and no per-caller variance sums.
static void run_tier1_batch(TfheAmdContext *l, const std::vector<Tier1Req *> &batch, double *ms,
                            const double *d_var) {
    for (const Tier1Req *q : batch)
        if (q->gate != batch[0]->gate) {
            run_tier1_mixed(l, batch, ms, d_var);
            return;
        }
    Tier1Clock::time_point t = Tier1Clock::now();
    const int gate = batch[0]->gate, n = (int)batch.size();
    const bool mux = gate == TFHE_GATE_MUX;
    // shallow copies of the samples: the a pointers and b values (taken before anything is written,
    // so a result may alias an input of its own call)
    std::vector<LweSample> rec((size_t)4 * n);
    LweSample *ra = rec.data(), *rb = ra + n, *rc3 = rb + n, *rr = rc3 + n;
    for (int i = 0; i < n; ++i) {
        const Tier1Req *q = batch[i];
        ra[i].a = q->a->a; ra[i].b = q->a->b;
        rb[i].a = q->b->a; rb[i].b = q->b->b;
        if (mux) { rc3[i].a = q->c->a; rc3[i].b = q->c->b; }
        rr[i].a = q->r->a;
    }
    auto rows = [](LweSample *x) {
        return TfheAmdRows{reinterpret_cast<char *>(x), sizeof(LweSample), offsetof(LweSample, a),
                           offsetof(LweSample, b), offsetof(LweSample, current_variance)};
    };
    const TfheAmdRows res = rows(rr), in[3] = {rows(ra), rows(rb), rows(rc3)};
    ms[1] += ms_since(t);
    const int rc = tfhe_amd_internal_gate_batch_rows(l, gate, n, &res, in, mux ? 3 : 2, d_var);
    ms[2] += ms_since(t);
    for (int i = 0; i < n; ++i) {
        Tier1Req *q = batch[i];
        q->rc = rc;
        if (rc != TFHE_AMD_OK) continue;
        q->r->b = rr[i].b;
        q->r->current_variance = rr[i].current_variance;
    }
    ms[4] += ms_since(t);
}

static void gate1(int gate, LweSample *r, const LweSample *a, const LweSample *b, const LweSample *c,
                  const TFheGateBootstrappingCloudKeySet *bk) {
    if (!coalesce_enabled()) {
        TfheAmdContext *l = lane_for(bk->bkFFT, nullptr);
        check(tfhe_amd_gate_batch_host(l, gate, 1, r->a, &r->b, a->a, &a->b, b->a, &b->b, c ? c->a : nullptr,
                                       c ? &c->b : nullptr),
              "gate");
        std::vector<int32_t> u;   // every gate ends in lweKeySwitch (boot-gates.cu:98-448)
        ks_input_of_last(l, 1, gate == TFHE_GATE_MUX ? 2 : 1, u);
        r->current_variance = ks_variance(bk->bkFFT->ks, u.data());
        return;
    }
    std::shared_ptr<KeyEntry> e = entry_for(bk->bkFFT, nullptr);
    Coalescer &q = e->q;
    Tier1Req req;
    req.gate = gate;
    req.r = r;
    req.a = a;
    req.b = b;
    req.c = c;
    std::unique_lock<std::mutex> lk(q.mu);
    if (q.window_us < 0) q.window_us = kWindowFloorUs;
    q.inside += 1;
    if (q.returning > 0) q.returning -= 1;
    q.pending.push_back(&req);
    // a collecting leader waits for every expected caller: wake it only when this arrival completes
    // the set (not once per arrival: with 64 callers on a 16-CPU share those wake-ups cost as much
    // as the batch's own host work)
    if (q.collecting && (int)q.pending.size() >= q.inside - q.in_flight + q.returning) q.arrive_cv.notify_all();
    // a free lane and no leader collecting: the oldest pending request's thread is asked to lead
    auto appoint = [&] {
        if (!q.collecting && q.running < kQueueLanes && !q.pending.empty() && q.pending.front() != &req)
            q.pending.front()->wake(false);
    };
    for (;;) {
        if (!req.taken && !q.collecting && q.running < kQueueLanes) break;   // lead the next batch
        lk.unlock();
        {
            std::unique_lock<std::mutex> rl(req.m);
            req.cv.wait(rl, [&] { return req.signaled; });
            req.signaled = false;
            if (req.done) break;
        }
        lk.lock();
    }
    if (!req.done) {
        // this thread leads the next batch, on a free lane
        int li = 0;
        while (q.lane_busy[li]) ++li;
        q.lane_busy[li] = true;
        q.running += 1;
        q.collecting = true;
        // stragglers: every thread inside a call and not in a running batch enqueues first, and so
        // do the callers the last batch released (an OpenMP team's threads come straight back with
        // their next gate): without them a team of T threads splits into alternating partial
        // batches instead of one batch of T
        auto all_in = [&] { return (int)q.pending.size() >= q.inside - q.in_flight + q.returning; };
        double bms[5] = {0, 0, 0, 0, 0};
        // merge instead of overlap: while the other lane's batch runs and both together would still
        // hold at most one ciphertext per CU, a second launch beside it only shares its CUs (two
        // latency-class launches of 31 run 2.15 ms each; one of 62 about 1.8), so wait for that batch
        // and take its callers' next gates too
        if (q.in_flight > 0 && (int)q.pending.size() + q.in_flight <= q.merge_limit) {
            const auto t0 = std::chrono::steady_clock::now();
            q.arrive_cv.wait(lk, [&] { return q.in_flight == 0; });
            bms[0] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        }
        if (!all_in() && q.window_us > 0) {
            const auto t0 = std::chrono::steady_clock::now();
            const bool ok = q.arrive_cv.wait_for(lk, std::chrono::duration<double, std::micro>(q.window_us), all_in);
            if (ok) {
                const double w = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                q.wait_avg_us = q.wait_avg_us > 0 ? 0.8 * q.wait_avg_us + 0.2 * w : w;
                q.window_us = std::min(1000.0, std::max(kWindowFloorUs, 4.0 * q.wait_avg_us + 20.0));
            } else {
                q.window_us = std::max(kWindowFloorUs, 0.75 * q.window_us);
                q.returning = 0;   // the released callers did not come back: stop expecting them
            }
            bms[0] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        }
        q.collecting = false;
        std::vector<Tier1Req *> batch;
        batch.swap(q.pending);
        for (Tier1Req *x : batch) x->taken = true;
        q.in_flight += (int)batch.size();
        if (q.running > 1) q.overlapped += 1;
        lk.unlock();
        // the queue's own lanes (stream + scratch), not the leader thread's: a thread that only
        // ever enqueues needs no lane, and leaders change from batch to batch
        TfheAmdContext *l;
        {
            std::lock_guard<std::mutex> lg(e->mu);
            if (!e->qlane[li]) e->qlane[li] = tfhe_amd_context_lane(e->primary);
            l = e->qlane[li];
        }
        if (!l) die_dramatically("tfhe_amd: cannot create the Tier-1 queue's GPU lane");
        const double *d_var = ks_variance_table(bk);
        if (!d_var) die_dramatically("tfhe_amd: cannot upload the key-switching key's row variances");
        run_tier1_batch(l, batch, bms, d_var);
        lk.lock();
        for (int k = 0; k < 5; ++k) q.ms[k] += bms[k];
        const int n = (int)batch.size();
        q.in_flight -= n;
        q.inside -= n;       // every caller of the batch (the leader too) leaves now ...
        q.returning += n;    // ... and may come back with its next gate
        q.running -= 1;
        q.lane_busy[li] = false;
        q.batches += 1;
        q.gates += n;
        q.largest = std::max(q.largest, (long long)n);
        q.arrive_cv.notify_all();   // a collecting leader's expected count changed
        appoint();                  // this lane is free again
        lk.unlock();
        auto wl = std::make_shared<std::vector<Tier1Req *>>();
        for (Tier1Req *x : batch)
            if (x != &req) wl->push_back(x);
        for (int i = 0; i < (int)wl->size(); ++i) {
            (*wl)[i]->wl = wl;
            (*wl)[i]->wi = i;
        }
        for (int i = 0; i < 2 && i < (int)wl->size(); ++i) (*wl)[i]->wake(true);   // may return from here on
    } else {
        // done by another thread's batch, whose leader did this call's bookkeeping: pass the wake-up on
        const std::shared_ptr<std::vector<Tier1Req *>> wl = std::move(req.wl);
        for (int c = 2 * req.wi + 2; wl && c < 2 * req.wi + 4 && c < (int)wl->size(); ++c) (*wl)[c]->wake(true);
    }
    check(req.rc, "gate");   // result and current_variance were written by the batch
}

// Builds the key's Tier-1 device context (key upload + conversion, HIP initialisation, the
// queue's lane) now, so that the first gate call pays only its own latency.
EXPORT int tfhe_amd_tier1_prepare(const TFheGateBootstrappingCloudKeySet *bk) {
    if (!bk || !bk->bkFFT) return TFHE_AMD_E_ARG;
    std::shared_ptr<KeyEntry> e = entry_for(bk->bkFFT, nullptr);
    std::lock_guard<std::mutex> lk(e->mu);
    for (auto *&ql : e->qlane)
        if (!ql) ql = tfhe_amd_context_lane(e->primary);
    return e->qlane[0] && e->qlane[1] ? TFHE_AMD_OK : TFHE_AMD_E_HIP;
}

EXPORT int tfhe_amd_tier1_queue_stats(const TFheGateBootstrappingCloudKeySet *bk, long long *batches,
                                      long long *gates, long long *largest, int reset) {
    if (!bk || !bk->bkFFT) return TFHE_AMD_E_ARG;
    std::shared_ptr<KeyEntry> e;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_reg.find(bk->bkFFT);
        if (it != g_reg.end()) e = it->second;
    }
    long long b = 0, g = 0, m = 0;
    if (e) {
        std::lock_guard<std::mutex> lk(e->q.mu);
        b = e->q.batches; g = e->q.gates; m = e->q.largest;
        if (reset) e->q.batches = e->q.gates = e->q.largest = 0;
    }
    if (batches) *batches = b;
    if (gates) *gates = g;
    if (largest) *largest = m;
    return TFHE_AMD_OK;
}

EXPORT int tfhe_amd_tier1_queue_times(const TFheGateBootstrappingCloudKeySet *bk, double *ms, int reset) {
    if (!bk || !bk->bkFFT) return TFHE_AMD_E_ARG;
    std::shared_ptr<KeyEntry> e;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_reg.find(bk->bkFFT);
        if (it != g_reg.end()) e = it->second;
    }
    double m[6] = {0, 0, 0, 0, 0, 0};
    if (e) {
        std::lock_guard<std::mutex> lk(e->q.mu);
        for (int k = 0; k < 5; ++k) {
            m[k] = e->q.ms[k];
            if (reset) e->q.ms[k] = 0;
        }
        m[5] = 0.0;   // (the callers no longer sum current_variance themselves)
    }
    if (ms)
        for (int k = 0; k < 6; ++k) ms[k] = m[k];
    return TFHE_AMD_OK;
}

EXPORT void bootsNAND(LweSample *r, const LweSample *a, const LweSample *b, const TFheGateBootstrappingCloudKeySet *bk) { gate1(TFHE_GATE_NAND, r, a, b, nullptr, bk); }
EXPORT void bootsOR(LweSample *r, const LweSample *a, const LweSample *b, const TFheGateBootstrappingCloudKeySet *bk) { gate1(TFHE_GATE_OR, r, a, b, nullptr, bk); }
EXPORT void bootsAND(LweSample *r, const LweSample *a, const LweSample *b, const TFheGateBootstrappingCloudKeySet *bk) { gate1(TFHE_GATE_AND, r, a, b, nullptr, bk); }
EXPORT void bootsXOR(LweSample *r, const LweSample *a, const LweSample *b, const TFheGateBootstrappingCloudKeySet *bk) { gate1(TFHE_GATE_XOR, r, a, b, nullptr, bk); }
EXPORT void bootsXNOR(LweSample *r, const LweSample *a, const LweSample *b, const TFheGateBootstrappingCloudKeySet *bk) { gate1(TFHE_GATE_XNOR, r, a, b, nullptr, bk); }
EXPORT void bootsNOR(LweSample *r, const LweSample *a, const LweSample *b, const TFheGateBootstrappingCloudKeySet *bk) { gate1(TFHE_GATE_NOR, r, a, b, nullptr, bk); }
EXPORT void bootsANDNY(LweSample *r, const LweSample *a, const LweSample *b, const TFheGateBootstrappingCloudKeySet *bk) { gate1(TFHE_GATE_ANDNY, r, a, b, nullptr, bk); }
EXPORT void bootsANDYN(LweSample *r, const LweSample *a, const LweSample *b, const TFheGateBootstrappingCloudKeySet *bk) { gate1(TFHE_GATE_ANDYN, r, a, b, nullptr, bk); }
EXPORT void bootsORNY(LweSample *r, const LweSample *a, const LweSample *b, const TFheGateBootstrappingCloudKeySet *bk) { gate1(TFHE_GATE_ORNY, r, a, b, nullptr, bk); }
EXPORT void bootsORYN(LweSample *r, const LweSample *a, const LweSample *b, const TFheGateBootstrappingCloudKeySet *bk) { gate1(TFHE_GATE_ORYN, r, a, b, nullptr, bk); }
EXPORT void bootsMUX(LweSample *r, const LweSample *a, const LweSample *b, const LweSample *c,
                     const TFheGateBootstrappingCloudKeySet *bk) {
    gate1(TFHE_GATE_MUX, r, a, b, c, bk);
}

// linear gates stay on the host (boot-gates.cu:242-267)
EXPORT void bootsNOT(LweSample *r, const LweSample *a, const TFheGateBootstrappingCloudKeySet *bk) {
    lweNegate(r, a, bk->params->in_out_params);
}
EXPORT void bootsCOPY(LweSample *r, const LweSample *a, const TFheGateBootstrappingCloudKeySet *bk) {
    lweCopy(r, a, bk->params->in_out_params);
}
EXPORT void bootsCONSTANT(LweSample *r, int value, const TFheGateBootstrappingCloudKeySet *bk) {
    const Torus32 MU = modSwitchToTorus32(1, 8);
    lweNoiselessTrivial(r, value ? MU : -MU, bk->params->in_out_params);
}

int tfhe_amd_internal_bk_coef(const TFheGateBootstrappingCloudKeySet *bk, int32_t *out) {
    if (!bk || !bk->bkFFT || !out) return TFHE_AMD_E_ARG;
    const std::vector<int32_t> &c = bkfft_of(bk->bkFFT)->bk_coef;
    memcpy(out, c.data(), sizeof(int32_t) * c.size());
    return TFHE_AMD_OK;
}

int tfhe_amd_internal_tier1_batch(const TFheGateBootstrappingCloudKeySet *bk, int gate, int B, int32_t *res_a,
                                  int32_t *res_b, const int32_t *a_a, const int32_t *a_b, const int32_t *b_a,
                                  const int32_t *b_b, const int32_t *c_a, const int32_t *c_b) {
    if (!bk || !bk->bkFFT) return TFHE_AMD_E_ARG;
    TfheAmdContext *l = lane_for(bk->bkFFT, nullptr);
    return tfhe_amd_gate_batch_host(l, gate, B, res_a, res_b, a_a, a_b, b_a, b_b, c_a, c_b);
}

// batched convenience over LweSample arrays: the engine gathers the records' rows straight into
// its pinned staging buffer and scatters the results back, pipelined in slices of one round, with
// current_variance computed on the device (tfhe_amd_internal_gate_batch_rows).  result may be the
// same array as an input.

EXPORT int tfhe_amd_boots_batch(int gate, LweSample *result, const LweSample *a, const LweSample *b,
                                const LweSample *c, int B, const TFheGateBootstrappingCloudKeySet *bk) {
    if (!bk || !bk->bkFFT || B < 0 || !result || !a || !b) return TFHE_AMD_E_ARG;
    if (B == 0) return TFHE_AMD_OK;
    if (gate == TFHE_GATE_MUX && !c) return TFHE_AMD_E_ARG;
    if (gate != TFHE_GATE_MUX) c = nullptr;
    TfheAmdContext *l = lane_for(bk->bkFFT, nullptr);
    const double *d_var = ks_variance_table(bk);
    if (!d_var) return TFHE_AMD_E_HIP;
    auto rows = [](const LweSample *x) {
        return TfheAmdRows{reinterpret_cast<char *>(const_cast<LweSample *>(x)), sizeof(LweSample),
                           offsetof(LweSample, a), offsetof(LweSample, b), offsetof(LweSample, current_variance)};
    };
    const TfheAmdRows res = rows(result), in[3] = {rows(a), rows(b), c ? rows(c) : rows(a)};
    return tfhe_amd_internal_gate_batch_rows(l, gate, B, &res, in, c ? 3 : 2, d_var);
}
