// tier1_rate.cpp — Tier-1 gate throughput from OpenMP teams (the reference's
// callers enter single gates from `#pragma omp parallel for` loops, Cipher.cpp:83-120,
// cloud.cpp:389-395).  Built against include/ + libtfhe_amd only (tests/callers/Makefile).
//
// A pool of P encrypted input pairs; every gate is bootsNAND(pool[i]) or, for odd i in the
// threaded runs, bootsNAND written in place over a copy of its first input (the result aliases
// an input, Cipher.cpp:306).  For each thread count T in argv (default 1 8 64) the team runs
// `per_thread` gates per thread (schedule static), timed; every output must equal the sequential
// result of the same gate word for word, and decrypt to the truth table.  The library's queue
// statistics (tfhe_amd_tier1_queue_stats) say how the calls were batched.  Run it with
// TFHE_AMD_TIER1_COALESCE=0 for the per-thread-lane path.
// Prints one JSON line; exit status 0 only when everything matched.
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <omp.h>
#include "tfhe/tfhe.h"
#include "tfhe_amd.h"

static bool same(const LweSample *x, const LweSample *y, int n) {
    return x->b == y->b && memcmp(x->a, y->a, sizeof(Torus32) * n) == 0;
}

int main(int argc, char **argv) {
    const int per_thread = argc > 1 ? atoi(argv[1]) : 8;
    std::vector<int> teams;
    for (int i = 2; i < argc; ++i) teams.push_back(atoi(argv[i]));
    if (teams.empty()) teams = {1, 8, 64};
    int maxT = 1;
    for (int t : teams) maxT = t > maxT ? t : maxT;
    const int P = maxT * per_thread;

    uint32_t seed[] = {314, 1592, 657};
    tfhe_random_generator_setSeed(seed, 3);
    TFheGateBootstrappingParameterSet *params = new_default_gate_bootstrapping_parameters(110);
    TFheGateBootstrappingSecretKeySet *key = new_random_gate_bootstrapping_secret_keyset(params);
    const TFheGateBootstrappingCloudKeySet *bk = &key->cloud;
    const LweParams *lp = params->in_out_params;
    const int dim = lp->n;

    std::vector<int> xa(P), xb(P);
    uint32_t s = 2024u;
    auto bit = [&]() { s = s * 1664525u + 1013904223u; return (int)(s >> 31); };
    LweSample *a = new_gate_bootstrapping_ciphertext_array(P, params);
    LweSample *b = new_gate_bootstrapping_ciphertext_array(P, params);
    for (int i = 0; i < P; i++) {
        xa[i] = bit(); xb[i] = bit();
        bootsSymEncrypt(&a[i], xa[i], key);
        bootsSymEncrypt(&b[i], xb[i], key);
    }
    LweSample *seq = new_gate_bootstrapping_ciphertext_array(P, params);
    LweSample *out = new_gate_bootstrapping_ciphertext_array(P, params);
    // warm-up (device context, key upload and conversion, lane) outside every timed region
    bootsNAND(&out[0], &a[0], &b[0], bk);
    double t0 = omp_get_wtime();
    for (int i = 0; i < P; i++) bootsNAND(&seq[i], &a[i], &b[i], bk);
    const double seq_s = omp_get_wtime() - t0;
    int truth_errors = 0;
    for (int i = 0; i < P; i++) truth_errors += bootsSymDecrypt(&seq[i], key) != !(xa[i] & xb[i]);

    std::string runs;
    int mismatches = 0;
    for (int T : teams) {
        const int n = T * per_thread;
        // untimed warm-up of the team (OpenMP threads created; per-thread lanes when the queue is off)
#pragma omp parallel for num_threads(T) schedule(static)
        for (int t = 0; t < T; t++) bootsNAND(&out[t], &a[t], &b[t], bk);
        for (int i = 0; i < n; i++) lweCopy(&out[i], &a[i], lp);
        tfhe_amd_tier1_queue_stats(bk, nullptr, nullptr, nullptr, 1);
        tfhe_amd_tier1_queue_times(bk, nullptr, 1);
        t0 = omp_get_wtime();
#pragma omp parallel for num_threads(T) schedule(static)
        for (int i = 0; i < n; i++) {
            if (i & 1) bootsNAND(&out[i], &out[i], &b[i], bk);   // in place: result aliases input a
            else bootsNAND(&out[i], &a[i], &b[i], bk);
        }
        const double dt = omp_get_wtime() - t0;
        long long nb = 0, ng = 0, big = 0;
        tfhe_amd_tier1_queue_stats(bk, &nb, &ng, &big, 1);
        double qms[6];
        tfhe_amd_tier1_queue_times(bk, qms, 1);
        int bad = 0;
        for (int i = 0; i < n; i++) bad += !same(&out[i], &seq[i], dim);
        mismatches += bad;
        char line[512];
        const double pb = nb ? 1.0 / nb : 0.0;   // per batch
        snprintf(line, sizeof line,
                 "%s{\"threads\": %d, \"gates\": %d, \"seconds\": %.4f, \"gates_per_s\": %.1f, \"mismatches\": %d, "
                 "\"batches\": %lld, \"mean_batch\": %.2f, \"largest_batch\": %lld, \"ms_per_batch\": {\"wait\": %.3f, "
                 "\"pack\": %.3f, \"device\": %.3f, \"mixed_variance\": %.3f, \"unpack\": %.3f}}",
                 runs.empty() ? "" : ", ", T, n, dt, n / dt, bad, nb, nb ? (double)ng / nb : 0.0, big, qms[0] * pb,
                 qms[1] * pb, qms[2] * pb, qms[3] * pb, qms[4] * pb);
        runs += line;
    }
    // mixed kinds: gate i is kind i mod 11 (the 10 binary gates and MUX), as threads of a real
    // program that sit in different parts of their circuits; the largest team, in place on odd i
    typedef void (*Gate2)(LweSample *, const LweSample *, const LweSample *, const TFheGateBootstrappingCloudKeySet *);
    const Gate2 g2[10] = {bootsNAND, bootsOR, bootsAND, bootsXOR, bootsXNOR, bootsNOR, bootsANDNY, bootsANDYN,
                          bootsORNY, bootsORYN};
    auto mixed = [&](int i, LweSample *r, const LweSample *x) {
        const int k = i % 11;
        if (k < 10) g2[k](r, x, &b[i], bk);
        else bootsMUX(r, x, &b[i], &a[(i + 1) % P], bk);
    };
    for (int i = 0; i < P; i++) mixed(i, &seq[i], &a[i]);
    const int T = maxT, n = maxT * per_thread;
    for (int i = 0; i < n; i++) lweCopy(&out[i], &a[i], lp);
    tfhe_amd_tier1_queue_stats(bk, nullptr, nullptr, nullptr, 1);
    tfhe_amd_tier1_queue_times(bk, nullptr, 1);
    t0 = omp_get_wtime();
#pragma omp parallel for num_threads(T) schedule(static)
    for (int i = 0; i < n; i++) {
        if (i & 1) mixed(i, &out[i], &out[i]);
        else mixed(i, &out[i], &a[i]);
    }
    const double dt_mixed = omp_get_wtime() - t0;
    long long nbm = 0, ngm = 0, bigm = 0;
    tfhe_amd_tier1_queue_stats(bk, &nbm, &ngm, &bigm, 1);
    double mms[6];
    tfhe_amd_tier1_queue_times(bk, mms, 1);
    const double pbm = nbm ? 1.0 / nbm : 0.0;
    int bad_mixed = 0;
    for (int i = 0; i < n; i++) bad_mixed += !same(&out[i], &seq[i], dim);
    mismatches += bad_mixed;
    const char *co = getenv("TFHE_AMD_TIER1_COALESCE");
    printf("{\"coalesce\": %s, \"pool\": %d, \"sequential_gates_per_s\": %.1f, \"truth_errors\": %d, "
           "\"mismatches\": %d, \"runs\": [%s], \"mixed_kinds\": {\"threads\": %d, \"gates\": %d, "
           "\"seconds\": %.4f, \"gates_per_s\": %.1f, \"mismatches\": %d, \"batches\": %lld, \"mean_batch\": %.2f, "
           "\"ms_per_batch\": {\"wait\": %.3f, \"pack\": %.3f, \"device\": %.3f, \"mixed_variance\": %.3f, \"unpack\": %.3f}}}\n",
           co && co[0] == '0' ? "false" : "true", P, P / seq_s, truth_errors, mismatches, runs.c_str(), T, n,
           dt_mixed, n / dt_mixed, bad_mixed, nbm, nbm ? (double)ngm / nbm : 0.0, mms[0] * pbm, mms[1] * pbm,
           mms[2] * pbm, mms[3] * pbm, mms[4] * pbm);
    delete_gate_bootstrapping_ciphertext_array(P, out);
    delete_gate_bootstrapping_ciphertext_array(P, seq);
    delete_gate_bootstrapping_ciphertext_array(P, b);
    delete_gate_bootstrapping_ciphertext_array(P, a);
    delete_gate_bootstrapping_secret_keyset(key);
    delete_gate_bootstrapping_parameters(params);
    return truth_errors || mismatches ? 1 : 0;
}
