// ref_driver.cpp — TEST INFRASTRUCTURE ONLY (our own code, not reference code).
// Flat-array C entry points that call the reference's OWN compiled leaf sources
// (gpuParallel/{numeric-functions,multiplication,lwe-functions,lwesamples,lwekey,
// lweparams,tgsw,tlwe,lwekeyswitch}.cu, built in place by oracle/build_ref.sh into
// oracle/_ref/libtfheref.so).
// Used only to generate the golden fixtures under tests/golden/ and, when the
// reference is present, to re-check the oracle directly.
#include <cstring>
#include <cstdint>
#include "tfhe_core.h"
#include "numeric_functions.h"
#include "polynomials.h"
#include "polynomials_arithmetic.h"
#include "lweparams.h"
#include "lwekey.h"
#include "lwesamples.h"
#include "lwe-functions.h"
#include "tlwe.h"
#include "tgsw.h"
#include "lwekeyswitch.h"
#include <vector>
EXPORT void tfhe_random_generator_setSeed(uint32_t* values, int size);  // numeric-functions.cu:16

extern "C" {

// multiplication.cu:72-77 torusPolynomialMultNaive (res = dig * poly mod X^N+1)
void ref_mult_naive(int32_t* res, const int32_t* dig, const int32_t* poly, int N) {
    IntPolynomial p1(N); TorusPolynomial p2(N), r(N);
    std::memcpy(p1.coefs, dig, N * 4); std::memcpy(p2.coefsT, poly, N * 4);
    torusPolynomialMultNaive(&r, &p1, &p2);
    std::memcpy(res, r.coefsT, N * 4);
}

// multiplication.cu:126-141 torusPolynomialMultKaratsuba
void ref_mult_karatsuba(int32_t* res, const int32_t* dig, const int32_t* poly, int N) {
    IntPolynomial p1(N); TorusPolynomial p2(N), r(N);
    std::memcpy(p1.coefs, dig, N * 4); std::memcpy(p2.coefsT, poly, N * 4);
    torusPolynomialMultKaratsuba(&r, &p1, &p2);
    std::memcpy(res, r.coefsT, N * 4);
}

// multiplication.cu:144-160 torusPolynomialAddMulRKaratsuba (res += dig*poly)
void ref_addmul_karatsuba(int32_t* res, const int32_t* dig, const int32_t* poly, int N) {
    IntPolynomial p1(N); TorusPolynomial p2(N), r(N);
    std::memcpy(p1.coefs, dig, N * 4); std::memcpy(p2.coefsT, poly, N * 4);
    std::memcpy(r.coefsT, res, N * 4);
    torusPolynomialAddMulRKaratsuba(&r, &p1, &p2);
    std::memcpy(res, r.coefsT, N * 4);
}

// numeric-functions.cu:60-66 / 72-77
void ref_modswitch_from(int32_t* out, const int32_t* x, int count, int Msize) {
    for (int i = 0; i < count; i++) out[i] = modSwitchFromTorus32(x[i], Msize);
}
int32_t ref_modswitch_to(int mu, int Msize) { return modSwitchToTorus32(mu, Msize); }

// numeric-functions.cu:16-19 + lwe-functions.cu:21-27 + 36-47: the reference RNG
// seeded with {seed...}, an LWE key of dimension n, then `count` encryptions
// of messages mu[i] with stdev alpha.  Outputs key[n], a[count][n], b[count].
void ref_lwe_keygen_encrypt(const uint32_t* seed, int nseed, int n, double alpha,
                            const int32_t* mu, int count,
                            int32_t* key_out, int32_t* a_out, int32_t* b_out) {
    tfhe_random_generator_setSeed(const_cast<uint32_t*>(seed), nseed);
    LweParams params(n, alpha, 1.0);
    LweKey key(&params);
    lweKeyGen(&key);
    std::memcpy(key_out, key.key, n * 4);
    LweSample s(&params);
    for (int c = 0; c < count; c++) {
        lweSymEncrypt(&s, mu[c], alpha, &key);
        std::memcpy(a_out + (size_t)c * n, s.a, n * 4);
        b_out[c] = s.b;
    }
}

// lwe-functions.cu:130-136, 145-151, 228-249, 276-291: op codes
// 0 NoiselessTrivial(mu) 1 AddTo 2 SubTo 3 AddMulTo(p) 4 SubMulTo(p) 5 Negate
void ref_lwe_op(int op, int n, int32_t* r_a, int32_t* r_b, const int32_t* s_a, int32_t s_b, int p) {
    LweParams params(n, 0.0, 1.0);
    LweSample r(&params), s(&params);
    std::memcpy(r.a, r_a, n * 4); r.b = *r_b;
    std::memcpy(s.a, s_a, n * 4); s.b = s_b;
    switch (op) {
    case 0: lweNoiselessTrivial(&r, p, &params); break;
    case 1: lweAddTo(&r, &s, &params); break;
    case 2: lweSubTo(&r, &s, &params); break;
    case 3: lweAddMulTo(&r, p, &s, &params); break;
    case 4: lweSubMulTo(&r, p, &s, &params); break;
    case 5: lweNegate(&r, &s, &params); break;
    }
    std::memcpy(r_a, r.a, n * 4); *r_b = r.b;
}

// tgsw.cu:7-29 TGswParams over tlwe.cu's TLweParams(N, k): the gadget h[] (l entries), the
// decomposition offset, kpl, Bg, halfBg, maskMod
void ref_tgsw_params(int l, int Bgbit, int N, int k, int32_t* h_out, uint32_t* offset_out, int32_t* ints_out) {
    TLweParams tp(N, k, 0.0, 1.0);
    TGswParams gp(l, Bgbit, &tp);
    for (int i = 0; i < l; i++) h_out[i] = gp.h[i];
    *offset_out = gp.offset;
    ints_out[0] = gp.kpl; ints_out[1] = gp.Bg; ints_out[2] = gp.halfBg; ints_out[3] = gp.maskMod;
}

// lwekeyswitch.cu:3-18: the row of ks0_raw that ks[i][j][h] addresses, for i < n, j < t,
// h < 2^basebit (pointer arithmetic on an unconstructed raw block: the constructor only
// builds the index arrays)
void ref_ksk_index(int n, int t, int basebit, int32_t* out) {
    const int base = 1 << basebit;
    std::vector<char> raw(sizeof(LweSample) * (size_t)n * t * base);
    LweSample* ks0 = reinterpret_cast<LweSample*>(raw.data());
    LweParams op(500, 0.0, 1.0);
    LweKeySwitchKey key(n, t, basebit, &op, ks0);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < t; j++)
            for (int h = 0; h < base; h++) out[((size_t)i * t + j) * base + h] = (int32_t)(key.ks[i][j] + h - ks0);
}

}
