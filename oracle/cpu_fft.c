/*
 * cpu_fft.c — TEST INFRASTRUCTURE ONLY: the optimized CPU baseline (bench.py's cpu_baseline
 * leg), never the product and never the parity checker (tfhe_oracle.c is).
 *
 * The reference CPU path links libtfhe-spqlios-avx (cpuParallel/compile.sh:1-2), whose
 * external product is a double-precision FFT over the negacyclic ring (tgsw-fft-operations.cu
 * :124-264; lagrangehalfc_impl.cu:95-117; fft_processor_fftw.cu:148-204).  spqlios is not
 * vendored in the reference and is not installed here or on the GPU box, so this file is an
 * optimized restatement of the same algorithm class, written for the host cores of the box:
 *
 *  * a polynomial a (N = 1024, real, mod X^N + 1) is folded to z_n = (a_n + i a_{n+512}) zeta^n
 *    (zeta = e^{i pi / 1024}) and transformed by a 512-point complex FFT: A(zeta w^k) at the 512
 *    roots of X^512 = i, which are roots of X^1024 + 1, so pointwise products are negacyclic
 *    products (the "half-size complex" trick spqlios and the reference's fft_processor use);
 *  * split re / im arrays, radix-2 stages whose inner loops run over contiguous twiddle rows
 *    (auto-vectorized: AVX2 4-wide / AVX-512 8-wide FMAs), forward Gentleman-Sande (natural in,
 *    bit-reversed out), inverse Cooley-Tukey (bit-reversed in, natural out): no permutation;
 *    the bootstrapping key is pre-transformed once with the 1/512 scale folded in;
 *  * results are rounded to the nearest integer mod 2^32 (the reference truncates,
 *    fft_processor_fftw.cu:177; the parity contract is the exact product),
 *    so outputs are Torus32-identical to the exact oracle while the FFT error stays < 1/2;
 *    cpufft_max_round_error() reports the largest |c - rint(c)| seen (tests assert < 1/4);
 *  * everything else (modswitch, test vector, rotation, decomposition, extraction, key switch,
 *    gate prologues) restates the same reference lines tfhe_oracle.c cites;
 *  * OpenMP over independent gates (the reference's cpuParallel runs gates concurrently from
 *    OpenMP threads too: Cipher.cpp:116-120, cloud.cpp:390-393).
 */
#include "cpu_fft.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define N 1024
#define H 512          /* complex points per transform */
#define NN 500
#define KPL 4

/* re / im of one spectrum; padded so that the 26 arrays the MAC streams (and the key's
 * 8 KB-strided rows) do not all map to the same cache sets */
typedef struct {
    double re[H], pad0[8], im[H], pad1[8];
} __attribute__((aligned(64))) Spec;

/* forward stage s (len = 512 >> s, half h = len / 2): twiddle e^{+2 pi i j / len}, j < h;
 * stored at offset H - len (rows 256 + 128 + ... fit in 512 entries) */
static double g_tw_re[H], g_tw_im[H];
static double g_twist_re[H], g_twist_im[H];   /* zeta^n */
static double g_untw_re[H], g_untw_im[H];     /* zeta^-n */
static int g_ready = 0;

static void init_tables(void) {
    if (g_ready) return;
    const long double PI = 3.14159265358979323846264338327950288L;
    for (int len = H; len >= 2; len >>= 1) {
        const int off = H - len;
        for (int j = 0; j < len / 2; j++) {
            const long double th = 2.0L * PI * (long double)j / (long double)len;
            g_tw_re[off + j] = (double)cosl(th);
            g_tw_im[off + j] = (double)sinl(th);
        }
    }
    for (int n = 0; n < H; n++) {
        const long double th = PI * (long double)n / (long double)N;
        g_twist_re[n] = (double)cosl(th);
        g_twist_im[n] = (double)sinl(th);
        g_untw_re[n] = (double)cosl(th);
        g_untw_im[n] = -(double)sinl(th);
    }
    g_ready = 1;
}
__attribute__((constructor)) static void cpufft_ctor(void) { init_tables(); }

/* forward DIF: natural -> bit-reversed, X[brv(k)] = sum_n x_n e^{+2 pi i n k / 512} */
static inline __attribute__((always_inline)) void fft_fwd(Spec *restrict x) {
    double *restrict re = x->re, *restrict im = x->im;
    for (int len = H; len >= 8; len >>= 1) {
        const int h = len >> 1;
        const double *restrict wr = g_tw_re + (H - len), *restrict wi = g_tw_im + (H - len);
        for (int b = 0; b < H; b += len) {
            double *restrict ur = re + b, *restrict ui = im + b, *restrict vr = re + b + h, *restrict vi = im + b + h;
            for (int j = 0; j < h; j++) {
                const double ar = ur[j], ai = ui[j], br = vr[j], bi = vi[j];
                const double dr = ar - br, di = ai - bi;
                ur[j] = ar + br;
                ui[j] = ai + bi;
                vr[j] = dr * wr[j] - di * wi[j];
                vi[j] = dr * wi[j] + di * wr[j];
            }
        }
    }
    /* len 4 (twiddles 1, i) and len 2 (twiddle 1), fused */
    for (int b = 0; b < H; b += 4) {
        const double r0 = re[b], r1 = re[b + 1], r2 = re[b + 2], r3 = re[b + 3];
        const double i0 = im[b], i1 = im[b + 1], i2 = im[b + 2], i3 = im[b + 3];
        const double s0r = r0 + r2, s0i = i0 + i2, s1r = r1 + r3, s1i = i1 + i3;
        const double d0r = r0 - r2, d0i = i0 - i2;
        const double d1r = -(i1 - i3), d1i = r1 - r3;   /* (x1 - x3) * i */
        re[b] = s0r + s1r; im[b] = s0i + s1i;
        re[b + 1] = s0r - s1r; im[b + 1] = s0i - s1i;
        re[b + 2] = d0r + d1r; im[b + 2] = d0i + d1i;
        re[b + 3] = d0r - d1r; im[b + 3] = d0i - d1i;
    }
}

/* inverse DIT: bit-reversed -> natural, x_n = sum_k X_k e^{-2 pi i n k / 512} (unscaled) */
static inline __attribute__((always_inline)) void fft_inv(Spec *restrict x) {
    double *restrict re = x->re, *restrict im = x->im;
    for (int b = 0; b < H; b += 4) {
        /* len 2 (twiddle 1) then len 4 (twiddles 1, -i) */
        const double r0 = re[b], r1 = re[b + 1], r2 = re[b + 2], r3 = re[b + 3];
        const double i0 = im[b], i1 = im[b + 1], i2 = im[b + 2], i3 = im[b + 3];
        const double a0r = r0 + r1, a0i = i0 + i1, a1r = r0 - r1, a1i = i0 - i1;
        const double a2r = r2 + r3, a2i = i2 + i3, a3r = r2 - r3, a3i = i2 - i3;
        const double t3r = a3i, t3i = -a3r;             /* a3 * (-i) */
        re[b] = a0r + a2r; im[b] = a0i + a2i;
        re[b + 2] = a0r - a2r; im[b + 2] = a0i - a2i;
        re[b + 1] = a1r + t3r; im[b + 1] = a1i + t3i;
        re[b + 3] = a1r - t3r; im[b + 3] = a1i - t3i;
    }
    for (int len = 8; len <= H; len <<= 1) {
        const int h = len >> 1;
        const double *restrict wr = g_tw_re + (H - len), *restrict wi = g_tw_im + (H - len);
        for (int b = 0; b < H; b += len) {
            double *restrict ur = re + b, *restrict ui = im + b, *restrict vr = re + b + h, *restrict vi = im + b + h;
            for (int j = 0; j < h; j++) {
                /* v * conj(w) */
                const double br = vr[j] * wr[j] + vi[j] * wi[j];
                const double bi = vi[j] * wr[j] - vr[j] * wi[j];
                const double ar = ur[j], ai = ui[j];
                ur[j] = ar + br;
                ui[j] = ai + bi;
                vr[j] = ar - br;
                vi[j] = ai - bi;
            }
        }
    }
}

/* fold + twist an integer polynomial into x, then transform */
static inline __attribute__((always_inline)) void poly_to_spec(Spec *restrict x, const int32_t *restrict a) {
    for (int n = 0; n < H; n++) {
        const double lo = (double)a[n], hi = (double)a[n + H];
        x->re[n] = lo * g_twist_re[n] - hi * g_twist_im[n];
        x->im[n] = lo * g_twist_im[n] + hi * g_twist_re[n];
    }
    fft_fwd(x);
}

/* rint(c) mod 2^32 for |c| < 2^82: the 1.5 * 2^84 shifter removes the multiple of 2^32, the
 * 1.5 * 2^52 shifter rounds the rest into the low mantissa word (exact except the rounding) */
static inline uint32_t torus_of(double c) {
    const double M1 = 0x1.8p84, M12 = 0x1.8p84 + 0x1.8p52;
    const double s = c + M1;
    const double t = s - M12;
    const double y = c - t;
    union { double d; uint64_t u; } v = {y};
    return (uint32_t)v.u;
}

/* c - rint(c) for |c| < 2^82 */
static inline double frac_dist(double c) {
    const double M1 = 0x1.8p84, M2 = 0x1.8p52;
    const double k = (c + M1) - M1;        /* c rounded to a multiple of 2^32 (exact) */
    const double d = c - k;                /* exact, |d| <= 2^31 */
    return d - ((d + M2) - M2);
}

/* inverse transform, untwist, round and ADD into acc (the tLweAddTo of tfhe_MuxRotate_FFT) */
static inline __attribute__((always_inline)) double spec_add_to_poly(uint32_t *restrict acc, Spec *restrict x) {
    fft_inv(x);
    double worst = 0.0;
    for (int n = 0; n < H; n++) {
        const double r = x->re[n] * g_untw_re[n] - x->im[n] * g_untw_im[n];
        const double i = x->re[n] * g_untw_im[n] + x->im[n] * g_untw_re[n];
        const uint32_t cr = torus_of(r), ci = torus_of(i);
        acc[n] += cr;
        acc[n + H] += ci;
        /* rounding distance: |c| < 2^52, so c - rint(c) is exact; rint by the 1.5 * 2^52
         * shifter on the part below 2^32 (the same exact operations as torus_of) */
        const double er = fabs(frac_dist(r)), ei = fabs(frac_dist(i));
        worst = er > worst ? er : worst;
        worst = ei > worst ? ei : worst;
    }
    return worst;
}

struct CpuFftKey {
    Spec *bk;                 /* [NN][KPL][2]: FFT(bk poly) / 512 */
    const int32_t *ksk;       /* [N][8][4][NN + 1] (borrowed) */
    double max_err;           /* largest rounding distance seen (racy max, diagnostics only) */
};

CpuFftKey *cpufft_key_create(const int32_t *bk, const int32_t *ksk) {
    init_tables();
    CpuFftKey *k = (CpuFftKey *)calloc(1, sizeof(CpuFftKey));
    if (!k) return NULL;
    k->ksk = ksk;
    if (posix_memalign((void **)&k->bk, 64, sizeof(Spec) * (size_t)NN * KPL * 2)) {
        free(k);
        return NULL;
    }
#pragma omp parallel for schedule(static)
    for (int t = 0; t < NN * KPL * 2; t++) {
        Spec *s = k->bk + t;
        poly_to_spec(s, bk + (size_t)t * N);
        for (int j = 0; j < H; j++) {
            s->re[j] *= 1.0 / H;
            s->im[j] *= 1.0 / H;
        }
    }
    return k;
}

void cpufft_key_free(CpuFftKey *k) {
    if (!k) return;
    free(k->bk);
    free(k);
}

double cpufft_max_round_error(const CpuFftKey *k) { return k ? k->max_err : 0.0; }

/* numeric-functions.cu:60-66 (wrapping uint64 sum: the result is always in [0, 2N)) */
static inline int modswitch_2N(int32_t phase) {
    const uint64_t interv = ((UINT64_C(1) << 63) / (uint64_t)(2 * N)) * 2;
    const uint64_t phase64 = ((uint64_t)(uint32_t)phase << 32) + interv / 2;
    return (int)(phase64 / interv);
}

typedef struct {
    Spec D[KPL], Y[2];
    int32_t dig[KPL][N];
    uint32_t tmp[2][N];
    uint32_t acc[2][N];
} Work;

/* tfhe_MuxRotate_FFT (lwe-bootstrapping-functions-fft.cu:105-185) with
 * tGswFFTExternMulToTLwe (tgsw-fft-operations.cu:124-264) in the FFT domain */
/* compiled twice: AVX-512F and the build's AVX2 baseline, picked at load time */
__attribute__((target_clones("avx512f", "default")))
static double cmux(uint32_t acc[2][N], const CpuFftKey *key, int i, int a, Work *w) {
    /* (X^a - 1) ACC (toruspolynomial-functions.cu:191-235), both polynomials */
    for (int c = 0; c < 2; c++) {
        const uint32_t *in = acc[c];
        uint32_t *out = w->tmp[c];
        if (a < N) {
            for (int j = 0; j < a; j++) out[j] = 0u - in[j - a + N] - in[j];
            for (int j = a; j < N; j++) out[j] = in[j - a] - in[j];
        } else {
            const int aa = a - N;
            for (int j = 0; j < aa; j++) out[j] = in[j - aa + N] - in[j];
            for (int j = aa; j < N; j++) out[j] = 0u - in[j - aa] - in[j];
        }
    }
    /* gadget decomposition (tgsw-functions.cu:322-351; offset of tgsw.cu:15-27) */
    const uint32_t off = 512u * ((1u << 22) + (1u << 12));
    for (int c = 0; c < 2; c++)
        for (int j = 0; j < N; j++) {
            const uint32_t buf = w->tmp[c][j] + off;
            w->dig[2 * c][j] = (int32_t)((buf >> 22) & 1023u) - 512;
            w->dig[2 * c + 1][j] = (int32_t)((buf >> 12) & 1023u) - 512;
        }
    for (int p = 0; p < KPL; p++) poly_to_spec(&w->D[p], w->dig[p]);
    const Spec *bki = key->bk + (size_t)i * KPL * 2;
    for (int c = 0; c < 2; c++) {
        double *restrict yr = w->Y[c].re, *restrict yi = w->Y[c].im;
        const double *restrict b0r = bki[0 * 2 + c].re, *restrict b0i = bki[0 * 2 + c].im;
        const double *restrict b1r = bki[1 * 2 + c].re, *restrict b1i = bki[1 * 2 + c].im;
        const double *restrict b2r = bki[2 * 2 + c].re, *restrict b2i = bki[2 * 2 + c].im;
        const double *restrict b3r = bki[3 * 2 + c].re, *restrict b3i = bki[3 * 2 + c].im;
        const double *restrict d0r = w->D[0].re, *restrict d0i = w->D[0].im;
        const double *restrict d1r = w->D[1].re, *restrict d1i = w->D[1].im;
        const double *restrict d2r = w->D[2].re, *restrict d2i = w->D[2].im;
        const double *restrict d3r = w->D[3].re, *restrict d3i = w->D[3].im;
        for (int k = 0; k < H; k++) {
            yr[k] = d0r[k] * b0r[k] - d0i[k] * b0i[k] + d1r[k] * b1r[k] - d1i[k] * b1i[k]
                  + d2r[k] * b2r[k] - d2i[k] * b2i[k] + d3r[k] * b3r[k] - d3i[k] * b3i[k];
            yi[k] = d0r[k] * b0i[k] + d0i[k] * b0r[k] + d1r[k] * b1i[k] + d1i[k] * b1r[k]
                  + d2r[k] * b2i[k] + d2i[k] * b2r[k] + d3r[k] * b3i[k] + d3i[k] * b3r[k];
        }
    }
    /* ACC += rint(ExtProd) (tLweAddTo, tlwe-functions.cu:170-192) */
    const double e0 = spec_add_to_poly(acc[0], &w->Y[0]);
    const double e1 = spec_add_to_poly(acc[1], &w->Y[1]);
    return e0 > e1 ? e0 : e1;
}

/* tfhe_bootstrap_woKS_FFT (lwe-bootstrapping-functions-fft.cu:1834-1870) with
 * tfhe_blindRotateAndExtract_FFT (:1408-1456) and extraction at index 0 (lwe.cu:41-56) */
static void bootstrap_woks(uint32_t *u_a, uint32_t *u_b, const CpuFftKey *key, int32_t mu, const int32_t *x_a,
                           int32_t x_b, Work *w) {
    uint32_t (*acc)[N] = w->acc;
    const int barb = modswitch_2N(x_b);
    /* ACC = (0, X^{2N - barb} (mu, ..., mu)) */
    const int e = (2 * N - barb) & (2 * N - 1);
    for (int j = 0; j < N; j++) {
        acc[0][j] = 0;
        acc[1][j] = ((j - e) & (2 * N - 1)) < N ? (uint32_t)mu : 0u - (uint32_t)mu;
    }
    double worst = 0.0;
    for (int i = 0; i < NN; i++) {
        const int a = modswitch_2N(x_a[i]);
        if (a == 0) continue;   /* :705 */
        const double err = cmux(acc, key, i, a, w);
        worst = err > worst ? err : worst;
    }
    if (worst > key->max_err) ((CpuFftKey *)key)->max_err = worst;
    u_a[0] = acc[0][0];
    for (int j = 1; j < N; j++) u_a[j] = 0u - acc[0][N - j];
    *u_b = acc[1][0];
}

/* lweKeySwitch (lwe-keyswitch-functions.cu:955-987 -> :101-127; layout lwekeyswitch.cu:3-18) */
static void keyswitch(int32_t *res_a, int32_t *res_b, const CpuFftKey *key, const uint32_t *u_a, uint32_t u_b) {
    uint32_t acc[NN + 1] __attribute__((aligned(64)));
    memset(acc, 0, sizeof(acc));
    acc[NN] = u_b;
    const uint32_t prec_offset = 1u << 15;
    for (int i = 0; i < N; i++) {
        const uint32_t aibar = u_a[i] + prec_offset;
        for (int j = 0; j < 8; j++) {
            const uint32_t aij = (aibar >> (30 - 2 * j)) & 3u;
            if (!aij) continue;
            const uint32_t *restrict row = (const uint32_t *)key->ksk + (((size_t)i * 8 + j) * 4 + aij) * (NN + 1);
            for (int k = 0; k <= NN; k++) acc[k] -= row[k];
        }
    }
    for (int k = 0; k < NN; k++) res_a[k] = (int32_t)acc[k];
    *res_b = (int32_t)acc[NN];
}

void cpufft_gate_batch(int B, int32_t c, int32_t sa, int32_t sb, int32_t *res_a, int32_t *res_b,
                       const int32_t *ca_a, const int32_t *ca_b, const int32_t *cb_a, const int32_t *cb_b,
                       const CpuFftKey *key, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    const int32_t mu = 1 << 29;   /* modSwitchToTorus32(1, 8) */
#pragma omp parallel
    {
        Work *w = NULL;
        if (posix_memalign((void **)&w, 64, sizeof(Work))) abort();
        int32_t t_a[NN];
        uint32_t u_a[N], u_b;
#pragma omp for schedule(dynamic, 1)
        for (int g = 0; g < B; g++) {
            /* gate prologue: (0, c) + sa ca + sb cb (boot-gates.cu:98-397) */
            const int32_t *xa = ca_a + (size_t)g * NN, *ya = cb_a + (size_t)g * NN;
            for (int k = 0; k < NN; k++) t_a[k] = (int32_t)((uint32_t)sa * (uint32_t)xa[k] + (uint32_t)sb * (uint32_t)ya[k]);
            const int32_t t_b = (int32_t)((uint32_t)c + (uint32_t)sa * (uint32_t)ca_b[g] + (uint32_t)sb * (uint32_t)cb_b[g]);
            bootstrap_woks(u_a, &u_b, key, mu, t_a, t_b, w);
            keyswitch(res_a + (size_t)g * NN, res_b + g, key, u_a, u_b);
        }
        free(w);
    }
}

void cpufft_woks_batch(int B, int32_t *out_a, int32_t *out_b, const CpuFftKey *key, int32_t mu,
                       const int32_t *x_a, const int32_t *x_b, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel
    {
        Work *w = NULL;
        if (posix_memalign((void **)&w, 64, sizeof(Work))) abort();
#pragma omp for schedule(dynamic, 1)
        for (int g = 0; g < B; g++)
            bootstrap_woks((uint32_t *)out_a + (size_t)g * N, (uint32_t *)out_b + g, key, mu, x_a + (size_t)g * NN,
                           x_b[g], w);
        free(w);
    }
}
