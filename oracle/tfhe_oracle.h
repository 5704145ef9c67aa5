/*
 * tfhe_oracle.h — TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * CPU restatement of the reference's gate-bootstrapping hot path
 * (toufique-morshed/CPU-GPU-TFHE, gpuParallel/ = vendored TFHE CPU path that
 * cpuParallel links as libtfhe-spqlios-avx).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load liboracle.so.
 *
 * Parity pinning:
 *   - the exact negacyclic product (multiplication.cu:64-77 torusPolynomialMultNaive_aux)
 *     and modSwitchFromTorus32/ToTorus32 (numeric-functions.cu:60-77) are pinned against
 *     the reference's own sources compiled in this container (oracle/build_ref.sh ->
 *     oracle/_ref/libtfheref.so) through committed fixtures in tests/golden/;
 *   - LWE-level ops (lweNoiselessTrivial/AddTo/SubTo/AddMulTo, lwe-functions.cu) are
 *     pinned the same way;
 *   - the remaining steps (rotation, gadget decomposition, extraction, key switch) are
 *     restatements cited line by line and checked by decryption truth tables; there is
 *     no reference golden vector for them ("parity partial").
 *
 * Layouts (canonical coefficient domain, int32 little endian):
 *   BK  : int32 [n=500][kpl=4][k+1=2][N=1024]   (TGswSample.all_sample[p].a[c].coefsT)
 *   KSK : int32 [N=1024][t=8][base=4][n+1=501]  (ks[i][j][h] = {a[500], b})
 */
#ifndef TFHE_ORACLE_H
#define TFHE_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORC_N = 1024, ORC_n = 500, ORC_k = 1, ORC_l = 2, ORC_Bgbit = 10, ORC_kpl = 4,
    ORC_ks_t = 8, ORC_ks_basebit = 2, ORC_ks_base = 4
};

/* gate codes shared with the product's C-ABI (include/tfhe_amd.h) */
enum {
    ORC_GATE_NAND = 0, ORC_GATE_OR, ORC_GATE_AND, ORC_GATE_XOR, ORC_GATE_XNOR,
    ORC_GATE_NOR, ORC_GATE_ANDNY, ORC_GATE_ANDYN, ORC_GATE_ORNY, ORC_GATE_ORYN,
    ORC_GATE_MUX
};

int32_t orc_modSwitchToTorus32(int mu, int Msize);
int     orc_modSwitchFromTorus32(int32_t phase, int Msize);

void orc_mul_by_xai(int32_t *out, int a, const int32_t *in);
void orc_mul_by_xai_minus_one(int32_t *out, int a, const int32_t *in);
void orc_decompose(int32_t *dec /*[l][N]*/, const int32_t *sample /*[N]*/);

/* res += dig * poly (negacyclic, exact, mod 2^32); schoolbook (definition) */
void orc_negacyclic_addmul_naive(int32_t *res, const int32_t *dig, const int32_t *poly);
/* same via the 2-prime CRT NTT */
void orc_negacyclic_addmul_ntt(int32_t *res, const int32_t *dig, const int32_t *poly);

/* A key handle: borrows bk/ksk (caller keeps them alive); use_ntt=1 precomputes the
 * NTT-domain BK (the CPU baseline path), use_ntt=0 keeps the schoolbook definition. */
typedef struct OrcKey OrcKey;
OrcKey *orc_key_create(const int32_t *bk, const int32_t *ksk, int use_ntt);
void    orc_key_free(OrcKey *key);

/* accum <- ExtProd(bk_i, (X^a - 1) accum) + accum for key index i */
void orc_mux_rotate(int32_t *accum /*[2][N]*/, const OrcKey *key, int i, int barai);
/* accum <- ExtProd(bk_i, accum) (no rotation) */
void orc_external_product(int32_t *accum /*[2][N]*/, const OrcKey *key, int i);

void orc_blind_rotate(int32_t *accum /*[2][N]*/, const OrcKey *key, const int32_t *bara, int n);

void orc_bootstrap_woKS(int32_t *out_a /*[N]*/, int32_t *out_b, const OrcKey *key, int32_t mu,
                        const int32_t *x_a /*[n]*/, int32_t x_b);
void orc_keyswitch(int32_t *res_a /*[n]*/, int32_t *res_b, const OrcKey *key,
                   const int32_t *u_a /*[N]*/, int32_t u_b);
void orc_bootstrap(int32_t *res_a, int32_t *res_b, const OrcKey *key,
                   int32_t mu, const int32_t *x_a, int32_t x_b);

/* one gate (incl. MUX: cc is the third input, ignored otherwise) */
void orc_gate(int gate, int32_t *res_a, int32_t *res_b,
              const int32_t *ca_a, int32_t ca_b, const int32_t *cb_a, int32_t cb_b,
              const int32_t *cc_a, int32_t cc_b, const OrcKey *key);

/* batched gates over B independent ciphertext tuples (SoA: a[B][n], b[B]),
 * OpenMP over ciphertexts with nthreads threads (<=0: OpenMP default) */
void orc_gate_batch(int gate, int B, int32_t *res_a, int32_t *res_b,
                    const int32_t *ca_a, const int32_t *ca_b,
                    const int32_t *cb_a, const int32_t *cb_b,
                    const int32_t *cc_a, const int32_t *cc_b,
                    const OrcKey *key, int nthreads);

/* woKS / KS batches (B samples) */
void orc_bootstrap_woKS_batch(int B, int32_t *out_a /*[B][N]*/, int32_t *out_b, const OrcKey *key,
                              int32_t mu, const int32_t *x_a, const int32_t *x_b, int nthreads);
void orc_keyswitch_batch(int B, int32_t *res_a, int32_t *res_b, const OrcKey *key,
                         const int32_t *u_a, const int32_t *u_b, int nthreads);

int orc_max_threads(void);

#ifdef __cplusplus
}
#endif
#endif
