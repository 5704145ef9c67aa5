/*
 * tfhe_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker and the CPU baseline,
 * never the product).  See tfhe_oracle.h for the pinning status.
 *
 * A plain-C restatement of the reference's CPU gate-bootstrapping path.  Every function
 * cites the reference file:line it restates (paths relative to the reference root,
 * gpuParallel/ = the vendored TFHE library that cpuParallel links).
 *
 * All Torus32 arithmetic is done on uint32_t (wrap-around mod 2^32, exactly the
 * int32 overflow behaviour the reference relies on) and cast at the end.
 *
 * The external product is computed EXACTLY (the semantics of multiplication.cu:64-77
 * summed over the kpl=4 rows, mod 2^32), either by schoolbook (use_ntt=0, the
 * definition) or by a 2-prime CRT negacyclic NTT (use_ntt=1, the fast CPU baseline).
 * The reference FFT path truncates its double result (fft_processor_fftw.cu:177); the
 * exact product is the parity contract.
 */
#include "tfhe_oracle.h"
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define N ORC_N
#define NN ORC_n

/* ------------------------------------------------------------------ numerics */

/* numeric-functions.cu:72-77 */
int32_t orc_modSwitchToTorus32(int mu, int Msize) {
    uint64_t interv = ((UINT64_C(1) << 63) / (uint64_t)Msize) * 2;
    uint64_t phase64 = (uint64_t)(int64_t)mu * interv;
    return (int32_t)(uint32_t)(phase64 >> 32);
}

/* numeric-functions.cu:60-66.  (phase << 32) + half_interval is computed in uint64_t and
 * WRAPS for phases just below 1 (x >= 2^32 - interv/2^33), which then map to 0 — the result
 * is always in [0, Msize) (pinned by tests/golden: -2^20 -> 0 at Msize 2048). */
int orc_modSwitchFromTorus32(int32_t phase, int Msize) {
    uint64_t interv = ((UINT64_C(1) << 63) / (uint64_t)Msize) * 2;
    uint64_t half_interval = interv / 2;
    uint64_t phase64 = ((uint64_t)(uint32_t)phase << 32) + half_interval;
    return (int)(phase64 / interv);
}

/* ------------------------------------------------------------ torus polys */

/* toruspolynomial-functions.cu:492-519  result = X^a * source, 0 <= a < 2N */
void orc_mul_by_xai(int32_t *out_, int a, const int32_t *in_) {
    uint32_t *out = (uint32_t *)out_;
    const uint32_t *in = (const uint32_t *)in_;
    if (a < N) {
        for (int i = 0; i < a; i++) out[i] = 0u - in[i - a + N];
        for (int i = a; i < N; i++) out[i] = in[i - a];
    } else {
        const int aa = a - N;
        for (int i = 0; i < aa; i++) out[i] = in[i - aa + N];
        for (int i = aa; i < N; i++) out[i] = 0u - in[i - aa];
    }
}

/* toruspolynomial-functions.cu:191-235  result = (X^a - 1) * source, 0 <= a < 2N
 * (a == 2N would take the a >= N branch with aa = N and yield 0). */
void orc_mul_by_xai_minus_one(int32_t *out_, int a, const int32_t *in_) {
    uint32_t *out = (uint32_t *)out_;
    const uint32_t *in = (const uint32_t *)in_;
    if (a < N) {
        for (int i = 0; i < a; i++) out[i] = 0u - in[i - a + N] - in[i];
        for (int i = a; i < N; i++) out[i] = in[i - a] - in[i];
    } else {
        const int aa = a - N;
        for (int i = 0; i < aa; i++) out[i] = in[i - aa + N] - in[i];
        for (int i = aa; i < N; i++) out[i] = 0u - in[i - aa] - in[i];
    }
}

/* tgsw-functions.cu:300-413 (scalar path :322-351, 391-392) with the parameters of
 * tgsw.cu:7-29: Bgbit=10, l=2, halfBg=512, maskMod=1023, offset = 512*(2^22+2^12). */
void orc_decompose(int32_t *dec, const int32_t *sample) {
    const uint32_t offset = 512u * ((1u << 22) + (1u << 12));
    for (int p = 0; p < ORC_l; ++p) {
        const int decal = 32 - (p + 1) * ORC_Bgbit;
        for (int j = 0; j < N; ++j) {
            uint32_t buf = (uint32_t)sample[j] + offset;
            uint32_t t = (buf >> decal) & 1023u;
            dec[p * N + j] = (int32_t)t - 512;
        }
    }
}

/* multiplication.cu:64-77 (torusPolynomialMultNaive_aux), accumulated as in
 * torusPolynomialAddMulR (multiplication.cu:144-177): res += dig * poly mod X^N+1 */
void orc_negacyclic_addmul_naive(int32_t *res_, const int32_t *dig, const int32_t *poly_) {
    uint32_t *res = (uint32_t *)res_;
    const uint32_t *poly = (const uint32_t *)poly_;
    for (int i = 0; i < N; i++) {
        uint32_t ri = 0;
        for (int j = 0; j <= i; j++) ri += (uint32_t)dig[j] * poly[i - j];
        for (int j = i + 1; j < N; j++) ri -= (uint32_t)dig[j] * poly[N + i - j];
        res[i] += ri;
    }
}

/* ------------------------------------------------------------ CRT NTT (exact) */
/* Two primes q < 2^30, q == 1 mod 2N; q0*q1 ~ 2^60 > 2 * 4*1024*512*2^31 = 2^53, so the
 * centred CRT lift recovers the exact integer external product. */
static const uint32_t Q[2] = {1073707009u, 1073698817u};
static uint32_t g_psi_br[2][N], g_psi_br_p[2][N];      /* psi^brv(k), Shoup companion */
static uint32_t g_ipsi_br[2][N], g_ipsi_br_p[2][N];    /* psi^-brv(k) */
static uint32_t g_ninv[2];
static uint32_t g_q0inv_mod_q1, g_q0inv_mod_q1_p;
static int g_tables_ready = 0;

static uint32_t powmod(uint32_t b, uint64_t e, uint32_t q) {
    uint64_t r = 1, x = b % q;
    while (e) { if (e & 1) r = r * x % q; x = x * x % q; e >>= 1; }
    return (uint32_t)r;
}
static unsigned brv10(unsigned x) {
    unsigned r = 0;
    for (int i = 0; i < 10; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}
static uint32_t shoup_p(uint32_t w, uint32_t q) { return (uint32_t)(((uint64_t)w << 32) / q); }

static void init_tables(void) {
    if (g_tables_ready) return;
    for (int s = 0; s < 2; s++) {
        const uint32_t q = Q[s];
        uint32_t psi = 0;
        for (uint32_t g = 2; g < 1000; g++) {
            uint32_t c = powmod(g, (q - 1) / (2 * N), q);
            if (powmod(c, N, q) == q - 1) { psi = c; break; }
        }
        uint32_t ipsi = powmod(psi, q - 2, q);
        for (int k = 0; k < N; k++) {
            g_psi_br[s][k] = powmod(psi, brv10(k), q);
            g_psi_br_p[s][k] = shoup_p(g_psi_br[s][k], q);
            g_ipsi_br[s][k] = powmod(ipsi, brv10(k), q);
            g_ipsi_br_p[s][k] = shoup_p(g_ipsi_br[s][k], q);
        }
        g_ninv[s] = powmod(N, q - 2, q);
    }
    g_q0inv_mod_q1 = powmod(Q[0] % Q[1], Q[1] - 2, Q[1]);
    g_q0inv_mod_q1_p = shoup_p(g_q0inv_mod_q1, Q[1]);
    g_tables_ready = 1;
}
__attribute__((constructor)) static void oracle_ctor(void) { init_tables(); }

/* a * w mod q for a < 2^32, w < q (Shoup); result in [0, q) */
static inline uint32_t mulmod_shoup(uint32_t a, uint32_t w, uint32_t wp, uint32_t q) {
    uint32_t qh = (uint32_t)(((uint64_t)a * wp) >> 32);
    uint32_t r = a * w - qh * q;
    return r >= q ? r - q : r;
}

/* forward negacyclic NTT (Cooley-Tukey, merged psi twist), natural -> bit-reversed */
static void ntt_fwd(uint32_t *a, int s) {
    const uint32_t q = Q[s];
    int t = N;
    for (int m = 1; m < N; m <<= 1) {
        t >>= 1;
        for (int i = 0; i < m; i++) {
            const uint32_t w = g_psi_br[s][m + i], wp = g_psi_br_p[s][m + i];
            uint32_t *x = a + 2 * i * t, *y = x + t;
            for (int j = 0; j < t; j++) {
                uint32_t u = x[j], v = mulmod_shoup(y[j], w, wp, q);
                uint32_t s0 = u + v;        s0 = s0 >= q ? s0 - q : s0;
                uint32_t d0 = u + q - v;    d0 = d0 >= q ? d0 - q : d0;
                x[j] = s0; y[j] = d0;
            }
        }
    }
}

/* inverse negacyclic NTT (Gentleman-Sande), bit-reversed -> natural, WITHOUT the 1/N
 * factor (it is folded into the NTT-domain key) */
static void ntt_inv(uint32_t *a, int s) {
    const uint32_t q = Q[s];
    int t = 1;
    for (int m = N; m > 1; m >>= 1) {
        const int h = m >> 1;
        for (int i = 0; i < h; i++) {
            const uint32_t w = g_ipsi_br[s][h + i], wp = g_ipsi_br_p[s][h + i];
            uint32_t *x = a + 2 * i * t, *y = x + t;
            for (int j = 0; j < t; j++) {
                uint32_t u = x[j], v = y[j];
                uint32_t s0 = u + v;        s0 = s0 >= q ? s0 - q : s0;
                uint32_t d0 = u + q - v;    d0 = d0 >= q ? d0 - q : d0;
                x[j] = s0; y[j] = mulmod_shoup(d0, w, wp, q);
            }
        }
        t <<= 1;
    }
}

static inline uint32_t to_mod(int32_t v, uint32_t q) {
    int64_t r = (int64_t)v % (int64_t)q;
    return (uint32_t)(r < 0 ? r + q : r);
}

/* centred CRT lift of (x0 mod q0, x1 mod q1) reduced mod 2^32 */
static inline uint32_t crt_torus(uint32_t x0, uint32_t x1) {
    const uint64_t M = (uint64_t)Q[0] * Q[1];
    uint32_t d = x1 + Q[1] - (x0 >= Q[1] ? x0 - Q[1] : x0);   /* x0 < q0 < 2 q1 */
    d = d >= Q[1] ? d - Q[1] : d;
    uint32_t h = mulmod_shoup(d, g_q0inv_mod_q1, g_q0inv_mod_q1_p, Q[1]);
    uint64_t X = (uint64_t)x0 + (uint64_t)Q[0] * h;            /* in [0, M) */
    if (X > M / 2) X -= M;                                     /* wraps: low 32 bits exact */
    return (uint32_t)X;
}

void orc_negacyclic_addmul_ntt(int32_t *res, const int32_t *dig, const int32_t *poly) {
    uint32_t A[2][N], B[2][N];
    for (int s = 0; s < 2; s++) {
        for (int j = 0; j < N; j++) { A[s][j] = to_mod(dig[j], Q[s]); B[s][j] = to_mod(poly[j], Q[s]); }
        ntt_fwd(A[s], s); ntt_fwd(B[s], s);
        for (int j = 0; j < N; j++)
            A[s][j] = (uint32_t)((uint64_t)A[s][j] * B[s][j] % Q[s] * g_ninv[s] % Q[s]);
        ntt_inv(A[s], s);
    }
    for (int j = 0; j < N; j++) res[j] = (int32_t)((uint32_t)res[j] + crt_torus(A[0][j], A[1][j]));
}

/* ------------------------------------------------------------------ keys */

struct OrcKey {
    const int32_t *bk;    /* [n][4][2][N] */
    const int32_t *ksk;   /* [N][8][4][n+1] */
    int use_ntt;
    uint32_t *bk_ntt;     /* [n][2 primes][4][2][N], scaled by 1/N */
};

/* BK preprocessing, the analogue of init_LweBootstrappingKeyFFT
 * (lwe-bootstrapping-functions-fft.cu:60-89 -> tGswToFFTConvert tgsw-fft-operations.cu:84-89) */
OrcKey *orc_key_create(const int32_t *bk, const int32_t *ksk, int use_ntt) {
    init_tables();
    OrcKey *k = (OrcKey *)calloc(1, sizeof(OrcKey));
    k->bk = bk; k->ksk = ksk; k->use_ntt = use_ntt;
    if (use_ntt && bk) {
        const size_t per_i = (size_t)2 * 4 * 2 * N;
        k->bk_ntt = (uint32_t *)malloc(sizeof(uint32_t) * per_i * NN);
#pragma omp parallel for schedule(static)
        for (int i = 0; i < NN; i++) {
            for (int s = 0; s < 2; s++)
                for (int p = 0; p < 4; p++)
                    for (int c = 0; c < 2; c++) {
                        uint32_t *dst = k->bk_ntt + i * per_i + ((size_t)(s * 4 + p) * 2 + c) * N;
                        const int32_t *src = bk + ((size_t)(i * 4 + p) * 2 + c) * N;
                        for (int j = 0; j < N; j++) dst[j] = to_mod(src[j], Q[s]);
                        ntt_fwd(dst, s);
                        for (int j = 0; j < N; j++) dst[j] = (uint32_t)((uint64_t)dst[j] * g_ninv[s] % Q[s]);
                    }
        }
    }
    return k;
}

void orc_key_free(OrcKey *k) {
    if (!k) return;
    free(k->bk_ntt);
    free(k);
}

/* ---------------------------------------------------------- external product */

/* tgsw-fft-operations.cu:124-264 tGswFFTExternMulToTLwe: decompose the k+1=2 accumulator
 * polys into kpl=4 digit polys (deca + i*l, :159-161), then out[c] = sum_p deca[p]*bk[p].a[c]
 * (tLweFFTAddMulRTo over p, :226-247) computed exactly, then back to the torus (:252). */
void orc_external_product(int32_t *accum, const OrcKey *key, int i) {
    int32_t dec[4][N];
    orc_decompose(dec[0], accum);          /* p = 0,1 : digits of a[0] */
    orc_decompose(dec[2], accum + N);      /* p = 2,3 : digits of a[1] = b */
    if (!key->use_ntt) {
        int32_t out[2][N];
        memset(out, 0, sizeof(out));
        const int32_t *bki = key->bk + (size_t)i * 4 * 2 * N;
        for (int p = 0; p < 4; p++)
            for (int c = 0; c < 2; c++)
                orc_negacyclic_addmul_naive(out[c], dec[p], bki + (p * 2 + c) * N);
        memcpy(accum, out, sizeof(out));
        return;
    }
    uint32_t D[4][N], O[2][2][N];
    const uint32_t *bki = key->bk_ntt + (size_t)i * 2 * 4 * 2 * N;
    for (int s = 0; s < 2; s++) {
        const uint32_t q = Q[s];
        for (int p = 0; p < 4; p++) {
            for (int j = 0; j < N; j++) { int32_t d = dec[p][j]; D[p][j] = d < 0 ? (uint32_t)(d + (int32_t)q) : (uint32_t)d; }
            ntt_fwd(D[p], s);
        }
        for (int c = 0; c < 2; c++) {
            const uint32_t *b0 = bki + ((size_t)(s * 4 + 0) * 2 + c) * N;
            const uint32_t *b1 = bki + ((size_t)(s * 4 + 1) * 2 + c) * N;
            const uint32_t *b2 = bki + ((size_t)(s * 4 + 2) * 2 + c) * N;
            const uint32_t *b3 = bki + ((size_t)(s * 4 + 3) * 2 + c) * N;
            for (int j = 0; j < N; j++) {
                uint64_t acc = (uint64_t)D[0][j] * b0[j] + (uint64_t)D[1][j] * b1[j]
                             + (uint64_t)D[2][j] * b2[j] + (uint64_t)D[3][j] * b3[j];
                O[s][c][j] = (uint32_t)(acc % q);
            }
            ntt_inv(O[s][c], s);
        }
    }
    for (int c = 0; c < 2; c++)
        for (int j = 0; j < N; j++) accum[c * N + j] = (int32_t)crt_torus(O[0][c][j], O[1][c][j]);
}

/* lwe-bootstrapping-functions-fft.cu:105-185 tfhe_MuxRotate_FFT:
 *   temp = (X^barai - 1) * ACC  (tLweMulByXaiMinusOne, tlwe-functions.cu:334-349)
 *   temp = BK_i (*) temp        (tGswFFTExternMulToTLwe)
 *   temp += ACC                 (tLweAddTo, tlwe-functions.cu:170-192)         */
void orc_mux_rotate(int32_t *accum, const OrcKey *key, int i, int barai) {
    int32_t tmp[2 * N];
    orc_mul_by_xai_minus_one(tmp, barai, accum);
    orc_mul_by_xai_minus_one(tmp + N, barai, accum + N);
    orc_external_product(tmp, key, i);
    for (int j = 0; j < 2 * N; j++) accum[j] = (int32_t)((uint32_t)tmp[j] + (uint32_t)accum[j]);
}

/* lwe-bootstrapping-functions-fft.cu:676-737 tfhe_blindRotate_FFT: skip bara_i == 0 (:705) */
void orc_blind_rotate(int32_t *accum, const OrcKey *key, const int32_t *bara, int n) {
    for (int i = 0; i < n; i++) {
        const int barai = bara[i];
        if (barai == 0) continue;
        orc_mux_rotate(accum, key, i, barai);
    }
}

/* lwe-bootstrapping-functions-fft.cu:1834-1870 tfhe_bootstrap_woKS_FFT
 *  -> :1408-1456 tfhe_blindRotateAndExtract_FFT -> lwe.cu:41-56 / 227-237 (index 0) */
void orc_bootstrap_woKS(int32_t *out_a, int32_t *out_b, const OrcKey *key, int32_t mu,
                        const int32_t *x_a, int32_t x_b) {
    const int Nx2 = 2 * N;
    int32_t bara[NN];
    const int barb = orc_modSwitchFromTorus32(x_b, Nx2);
    for (int i = 0; i < NN; i++) bara[i] = orc_modSwitchFromTorus32(x_a[i], Nx2);
    int32_t testvect[N], acc[2 * N];
    for (int i = 0; i < N; i++) testvect[i] = mu;
    /* testvectbis = X^{2N-barb} * v, or a copy when barb == 0 (:1427-1428); barb == 2N
     * gives the exponent 0 and therefore also the copy */
    if (barb != 0) orc_mul_by_xai(acc + N, Nx2 - barb, testvect);
    else memcpy(acc + N, testvect, sizeof(testvect));
    memset(acc, 0, N * sizeof(int32_t));            /* tLweNoiselessTrivial tlwe-functions.cu:130-138 */
    orc_blind_rotate(acc, key, bara, NN);
    /* tLweExtractLweSampleIndex(index 0), lwe.cu:41-56 */
    out_a[0] = acc[0];
    for (int j = 1; j < N; j++) out_a[j] = (int32_t)(0u - (uint32_t)acc[N - j]);
    *out_b = acc[N + 0];
}

/* lwe-keyswitch-functions.cu:955-987 lweKeySwitch -> :101-127 lweKeySwitchTranslate_fromArray
 * KSK layout ks[i][j][h] (lwekeyswitch.cu:3-18), basebit=2, t=8, prec_offset = 2^(32-17) */
void orc_keyswitch(int32_t *res_a, int32_t *res_b, const OrcKey *key, const int32_t *u_a, int32_t u_b) {
    const int basebit = ORC_ks_basebit, t = ORC_ks_t, base = 1 << basebit;
    const uint32_t prec_offset = 1u << (32 - (1 + basebit * t));
    const uint32_t mask = base - 1;
    uint32_t acc[NN + 1];
    memset(acc, 0, sizeof(acc));
    acc[NN] = (uint32_t)u_b;                    /* lweNoiselessTrivial(result, sample->b) */
    for (int i = 0; i < N; i++) {
        const uint32_t aibar = (uint32_t)u_a[i] + prec_offset;
        for (int j = 0; j < t; j++) {
            const uint32_t aij = (aibar >> (32 - (j + 1) * basebit)) & mask;
            if (aij != 0) {                     /* lweSubTo(result, &ks[i][j][aij]) */
                const int32_t *row = key->ksk + (((size_t)i * t + j) * base + aij) * (NN + 1);
                for (int k = 0; k <= NN; k++) acc[k] -= (uint32_t)row[k];
            }
        }
    }
    for (int k = 0; k < NN; k++) res_a[k] = (int32_t)acc[k];
    *res_b = (int32_t)acc[NN];
}

/* lwe-bootstrapping-functions-fft.cu:1884-1910 tfhe_bootstrap_FFT = woKS + KS */
void orc_bootstrap(int32_t *res_a, int32_t *res_b, const OrcKey *key, int32_t mu,
                   const int32_t *x_a, int32_t x_b) {
    int32_t u_a[N], u_b;
    orc_bootstrap_woKS(u_a, &u_b, key, mu, x_a, x_b);
    orc_keyswitch(res_a, res_b, key, u_a, u_b);
}

/* ------------------------------------------------------------------ gates */

/* gate prologue constants, boot-gates.cu:98-397: tmp = (0, c) + sa*ca + sb*cb */
static void gate_coeffs(int gate, int32_t *c, int *sa, int *sb) {
    switch (gate) {
    case ORC_GATE_NAND:  *c = orc_modSwitchToTorus32(1, 8);  *sa = -1; *sb = -1; break; /* :98-116 */
    case ORC_GATE_OR:    *c = orc_modSwitchToTorus32(1, 8);  *sa = 1;  *sb = 1;  break; /* :124-142 */
    case ORC_GATE_AND:   *c = orc_modSwitchToTorus32(-1, 8); *sa = 1;  *sb = 1;  break; /* :150-182 */
    case ORC_GATE_XOR:   *c = orc_modSwitchToTorus32(1, 4);  *sa = 2;  *sb = 2;  break; /* :190-208 */
    case ORC_GATE_XNOR:  *c = orc_modSwitchToTorus32(-1, 4); *sa = -2; *sb = -2; break; /* :216-234 */
    case ORC_GATE_NOR:   *c = orc_modSwitchToTorus32(-1, 8); *sa = -1; *sb = -1; break; /* :275-293 */
    case ORC_GATE_ANDNY: *c = orc_modSwitchToTorus32(-1, 8); *sa = -1; *sb = 1;  break; /* :301-321 */
    case ORC_GATE_ANDYN: *c = orc_modSwitchToTorus32(-1, 8); *sa = 1;  *sb = -1; break; /* :325-345 */
    case ORC_GATE_ORNY:  *c = orc_modSwitchToTorus32(1, 8);  *sa = -1; *sb = 1;  break; /* :349-369 */
    case ORC_GATE_ORYN:  *c = orc_modSwitchToTorus32(1, 8);  *sa = 1;  *sb = -1; break; /* :373-397 */
    default: abort();
    }
}

/* lweNoiselessTrivial + lweAddTo/lweSubTo/lweAddMulTo/lweSubMulTo (lwe-functions.cu:130-282) */
static void lwe_combine(int32_t *t_a, int32_t *t_b, int32_t c, int sa, const int32_t *ca_a, int32_t ca_b,
                        int sb, const int32_t *cb_a, int32_t cb_b) {
    for (int i = 0; i < NN; i++)
        t_a[i] = (int32_t)((uint32_t)sa * (uint32_t)ca_a[i] + (uint32_t)sb * (uint32_t)cb_a[i]);
    *t_b = (int32_t)((uint32_t)c + (uint32_t)sa * (uint32_t)ca_b + (uint32_t)sb * (uint32_t)cb_b);
}

void orc_gate(int gate, int32_t *res_a, int32_t *res_b,
              const int32_t *ca_a, int32_t ca_b, const int32_t *cb_a, int32_t cb_b,
              const int32_t *cc_a, int32_t cc_b, const OrcKey *key) {
    const int32_t MU = orc_modSwitchToTorus32(1, 8);
    int32_t t_a[NN], t_b;
    if (gate == ORC_GATE_MUX) {
        /* boot-gates.cu:407-448: u1 = woKS(AND(a,b)), u2 = woKS(AND(not a, c)),
         * res = KS((0,1/8) + u1 + u2) */
        const int32_t AndConst = orc_modSwitchToTorus32(-1, 8);
        const int32_t MuxConst = orc_modSwitchToTorus32(1, 8);
        int32_t u1_a[N], u1_b, u2_a[N], u2_b;
        lwe_combine(t_a, &t_b, AndConst, 1, ca_a, ca_b, 1, cb_a, cb_b);
        orc_bootstrap_woKS(u1_a, &u1_b, key, MU, t_a, t_b);
        lwe_combine(t_a, &t_b, AndConst, -1, ca_a, ca_b, 1, cc_a, cc_b);
        orc_bootstrap_woKS(u2_a, &u2_b, key, MU, t_a, t_b);
        for (int j = 0; j < N; j++) u1_a[j] = (int32_t)((uint32_t)u1_a[j] + (uint32_t)u2_a[j]);
        u1_b = (int32_t)((uint32_t)MuxConst + (uint32_t)u1_b + (uint32_t)u2_b);
        orc_keyswitch(res_a, res_b, key, u1_a, u1_b);
        return;
    }
    int32_t c; int sa, sb;
    gate_coeffs(gate, &c, &sa, &sb);
    lwe_combine(t_a, &t_b, c, sa, ca_a, ca_b, sb, cb_a, cb_b);
    orc_bootstrap(res_a, res_b, key, MU, t_a, t_b);
}

static void set_threads(int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
}

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void orc_gate_batch(int gate, int B, int32_t *res_a, int32_t *res_b,
                    const int32_t *ca_a, const int32_t *ca_b,
                    const int32_t *cb_a, const int32_t *cb_b,
                    const int32_t *cc_a, const int32_t *cc_b,
                    const OrcKey *key, int nthreads) {
    set_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
    for (int b = 0; b < B; b++) {
        orc_gate(gate, res_a + (size_t)b * NN, res_b + b,
                 ca_a + (size_t)b * NN, ca_b[b], cb_a + (size_t)b * NN, cb_b[b],
                 cc_a ? cc_a + (size_t)b * NN : NULL, cc_b ? cc_b[b] : 0, key);
    }
}

void orc_bootstrap_woKS_batch(int B, int32_t *out_a, int32_t *out_b, const OrcKey *key,
                              int32_t mu, const int32_t *x_a, const int32_t *x_b, int nthreads) {
    set_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
    for (int b = 0; b < B; b++)
        orc_bootstrap_woKS(out_a + (size_t)b * N, out_b + b, key, mu, x_a + (size_t)b * NN, x_b[b]);
}

void orc_keyswitch_batch(int B, int32_t *res_a, int32_t *res_b, const OrcKey *key,
                         const int32_t *u_a, const int32_t *u_b, int nthreads) {
    set_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
    for (int b = 0; b < B; b++)
        orc_keyswitch(res_a + (size_t)b * NN, res_b + b, key, u_a + (size_t)b * N, u_b[b]);
}
