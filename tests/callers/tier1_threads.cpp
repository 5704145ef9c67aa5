// tier1_threads.cpp — Tier-1 (single-sample TFHE C API) reentrancy and aliasing check, built
// against include/ + libtfhe_amd only (tests/callers/Makefile).  SURVEY.md §8(b): the
// reference's callers enter the gates from OpenMP threads (Cipher.cpp:116-120, cloud.cpp:390-393)
// and pass a result that aliases an input (Cipher.cpp:306, 387: bootsAND(t1, t1, t2)).
// Every gate of the API is evaluated on the same encrypted inputs three ways — sequentially,
// from 8 OpenMP threads at once, and in place — and the three results must be the same
// samples, word for word (the engine is deterministic); each must decrypt to its truth table.
// Then 16 short-lived std::threads each run one gate and exit: every exiting thread must give
// its lane (stream + scratch) back, so the key's lane count returns to what it was.
// Round 5: samples compare with current_variance bit for bit, and a mixed phase runs
// the units interleaved (consecutive calls of a thread are different kinds, MUX among them) from 8
// threads, so the coalescing queue's batches mix kinds and their current_variance comes from the
// mixed launch's device-side sum (tfhe_amd_internal_mixed_variance / k_ks_variance_rows), which
// must equal the variance of the same gate run alone.  argv[2] = "nonuniform": the key-switching
// key's row variances are made unequal before the first gate (the device sum's general form).
// Prints one JSON line; exit status 0 only when everything matched.
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <omp.h>
#include <thread>
#include "tfhe/tfhe.h"
#include "tfhe_amd.h"

typedef void (*Gate2)(LweSample *, const LweSample *, const LweSample *, const TFheGateBootstrappingCloudKeySet *);

struct Gate {
    const char *name;
    Gate2 f;
    int (*truth)(int, int);
};

static int t_nand(int a, int b) { return !(a & b); }
static int t_and(int a, int b) { return a & b; }
static int t_or(int a, int b) { return a | b; }
static int t_xor(int a, int b) { return a ^ b; }
static int t_xnor(int a, int b) { return !(a ^ b); }
static int t_nor(int a, int b) { return !(a | b); }
static int t_andny(int a, int b) { return (!a) & b; }
static int t_andyn(int a, int b) { return a & (!b); }
static int t_orny(int a, int b) { return (!a) | b; }
static int t_oryn(int a, int b) { return a | (!b); }

static bool same(const LweSample *x, const LweSample *y, int n) {
    return x->b == y->b && memcmp(x->a, y->a, sizeof(Torus32) * n) == 0 &&
           memcmp(&x->current_variance, &y->current_variance, sizeof(double)) == 0;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 32;   // samples per gate
    const Gate gates[] = {{"NAND", bootsNAND, t_nand},   {"AND", bootsAND, t_and},     {"OR", bootsOR, t_or},
                          {"XOR", bootsXOR, t_xor},      {"XNOR", bootsXNOR, t_xnor},  {"NOR", bootsNOR, t_nor},
                          {"ANDNY", bootsANDNY, t_andny}, {"ANDYN", bootsANDYN, t_andyn}, {"ORNY", bootsORNY, t_orny},
                          {"ORYN", bootsORYN, t_oryn}};
    const int ng = sizeof(gates) / sizeof(gates[0]);
    const int units = ng + 1;   // + MUX

    uint32_t seed[] = {314, 1592, 657};
    tfhe_random_generator_setSeed(seed, 3);
    TFheGateBootstrappingParameterSet *params = new_default_gate_bootstrapping_parameters(110);
    TFheGateBootstrappingSecretKeySet *key = new_random_gate_bootstrapping_secret_keyset(params);
    const TFheGateBootstrappingCloudKeySet *bk = &key->cloud;
    const LweParams *lp = params->in_out_params;
    const bool nonuniform = argc > 2 && strcmp(argv[2], "nonuniform") == 0;
    if (nonuniform) {   // unequal row variances, before the key's device tables exist
        LweSample *rows = bk->bkFFT->ks->ks0_raw;
        for (int r = 0; r < 1024 * 8 * 4; r++) rows[r].current_variance *= 1.0 + ((r * 37) % 11) * 1e-3;
    }
    const int dim = lp->n;

    std::vector<int> xa(n), xb(n), xc(n);
    uint32_t s = 12345u;
    auto bit = [&]() { s = s * 1664525u + 1013904223u; return (int)(s >> 31); };
    LweSample *a = new_gate_bootstrapping_ciphertext_array(n, params);
    LweSample *b = new_gate_bootstrapping_ciphertext_array(n, params);
    LweSample *c = new_gate_bootstrapping_ciphertext_array(n, params);
    for (int i = 0; i < n; i++) {
        xa[i] = bit(); xb[i] = bit(); xc[i] = bit();
        bootsSymEncrypt(&a[i], xa[i], key);
        bootsSymEncrypt(&b[i], xb[i], key);
        bootsSymEncrypt(&c[i], xc[i], key);
    }
    const int total = units * n;
    LweSample *seq = new_gate_bootstrapping_ciphertext_array(total, params);
    LweSample *par = new_gate_bootstrapping_ciphertext_array(total, params);
    LweSample *ali = new_gate_bootstrapping_ciphertext_array(total, params);
    LweSample *mix = new_gate_bootstrapping_ciphertext_array(total, params);

    auto run = [&](int k, LweSample *out) {
        const int g = k / n, i = k % n;
        if (g < ng) gates[g].f(out, &a[i], &b[i], bk);
        else bootsMUX(out, &a[i], &b[i], &c[i], bk);
    };
    double t0 = omp_get_wtime();
    for (int k = 0; k < total; k++) run(k, &seq[k]);
    double t1 = omp_get_wtime();
#pragma omp parallel for num_threads(8) schedule(dynamic, 1)
    for (int k = 0; k < total; k++) run(k, &par[k]);
    double t2 = omp_get_wtime();
    // in place: the result is the first input (even k) or the second / the MUX's c (odd k)
#pragma omp parallel for num_threads(4) schedule(dynamic, 1)
    for (int k = 0; k < total; k++) {
        const int g = k / n, i = k % n;
        LweSample *r = &ali[k];
        if (g < ng) {
            if (k & 1) { lweCopy(r, &b[i], lp); gates[g].f(r, &a[i], r, bk); }
            else { lweCopy(r, &a[i], lp); gates[g].f(r, r, &b[i], bk); }
        } else {
            lweCopy(r, &c[i], lp);
            bootsMUX(r, &a[i], &b[i], r, bk);
        }
    }
    // interleaved kinds: call q runs unit (q mod units) on sample (q / units), statically dealt
    // round-robin to 8 threads, so every batch the queue forms holds several kinds (MUX included)
#pragma omp parallel for num_threads(8) schedule(static, 1)
    for (int q = 0; q < total; q++) {
        const int k = (q % units) * n + q / units;
        run(k, &mix[k]);
    }
    // short-lived threads: one gate each, then exit
    const int lanes_before = tfhe_amd_tier1_lane_count(bk);
    int short_errors = 0;
    for (int t = 0; t < 16; t++) {
        LweSample *r = new_gate_bootstrapping_ciphertext_array(1, params);
        const int i = t % n;
        std::thread th([&] { bootsNAND(r, &a[i], &b[i], bk); });
        th.join();
        short_errors += !same(r, &seq[i], dim);   // gate 0 is NAND: seq[i] = NAND(a[i], b[i])
        delete_gate_bootstrapping_ciphertext_array(1, r);
    }
    const int lanes_after = tfhe_amd_tier1_lane_count(bk);
    int par_mismatch = 0, alias_mismatch = 0, mixed_mismatch = 0, truth_errors = 0, zero_variance = 0;
    for (int k = 0; k < total; k++) {
        const int g = k / n, i = k % n;
        par_mismatch += !same(&seq[k], &par[k], dim);
        alias_mismatch += !same(&seq[k], &ali[k], dim);
        mixed_mismatch += !same(&seq[k], &mix[k], dim);
        zero_variance += !(seq[k].current_variance > 0);
        const int want = g < ng ? gates[g].truth(xa[i], xb[i]) : (xa[i] ? xb[i] : xc[i]);
        truth_errors += bootsSymDecrypt(&seq[k], key) != want;
    }
    printf("{\"units\": %d, \"per_unit\": %d, \"threads\": 8, \"par_mismatch\": %d, \"alias_mismatch\": %d, "
           "\"mixed_mismatch\": %d, \"zero_variance\": %d, \"nonuniform_key\": %d, \"truth_errors\": %d, \"seq_ms_per_gate\": %.3f, \"par_ms_per_gate\": %.3f, \"lanes_before\": %d, "
           "\"lanes_after_short_threads\": %d, \"short_thread_errors\": %d}\n",
           units, n, par_mismatch, alias_mismatch, mixed_mismatch, zero_variance, (int)nonuniform, truth_errors, 1e3 * (t1 - t0) / total, 1e3 * (t2 - t1) / total,
           lanes_before, lanes_after, short_errors);
    delete_gate_bootstrapping_ciphertext_array(total, mix);
    delete_gate_bootstrapping_ciphertext_array(total, ali);
    delete_gate_bootstrapping_ciphertext_array(total, par);
    delete_gate_bootstrapping_ciphertext_array(total, seq);
    delete_gate_bootstrapping_ciphertext_array(n, c);
    delete_gate_bootstrapping_ciphertext_array(n, b);
    delete_gate_bootstrapping_ciphertext_array(n, a);
    delete_gate_bootstrapping_secret_keyset(key);
    delete_gate_bootstrapping_parameters(params);
    return par_mismatch || alias_mismatch || mixed_mismatch || zero_variance || truth_errors || short_errors ||
                   lanes_after != lanes_before
               ? 1
               : 0;
}
