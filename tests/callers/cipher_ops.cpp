// cipher_ops.cpp — drives the reference's own Cipher class (cpuParallel/Cipher.cpp, compiled
// unchanged by oracle/build_callers.sh) on top of libtfhe_amd, from the files the reference's
// cpuParallel/main.cpp writes (secret.key, cloud.key, cloud.data in the working directory).
// Cipher's static initialiser (Cipher.cpp:10-17) loads cloud.key before main runs.
//
// Prints one JSON line with the decrypted results of the reference's circuits:
//   a + b (operator+, Cipher.cpp ripple-carry with addBits), a - b (twosComplement + add),
//   a * b (operator*, shift-and-add; on the low 8 bits), minimum(a, b), a == b, a > b.
// `cipher_ops add32 A B`: BASELINE config 3 through the unchanged Cipher::operator+
// (Cipher.cpp:348-392, 5 gates per bit) on 32-bit operands encrypted here with
// bootsSymEncrypt under secret.key; prints {"a", "b", "sum", "seconds", "first_gate_seconds"}.
// `cipher_ops mul16 A B [threads]`: Cipher::operator* on 16-bit operands (see mul16 below).
// Integration tests only (tests/test_io.py::test_reference_callers_gpu,
// tests/test_configs_gpu.py::test_config3_cipher_operator_plus_32bit).
#include <cstdio>
#include <cstdlib>
#include <omp.h>
#include <string>

#include "Cipher.h"
#include "tfhe_amd.h"

static long decode(const Cipher &c, const TFheGateBootstrappingSecretKeySet *key) {
    long v = 0;
    for (int i = 0; i < c.numberOfBits; i++) v |= (long)bootsSymDecrypt(&c.data[i], key) << i;
    return v;
}

static int add32(const TFheGateBootstrappingSecretKeySet *key, long av, long bv) {
    const TFheGateBootstrappingParameterSet *params = Cipher::bk->params;
    const int bits = 32;
    LweSample *x = new_gate_bootstrapping_ciphertext_array(bits, params);
    LweSample *y = new_gate_bootstrapping_ciphertext_array(bits, params);
    for (int i = 0; i < bits; i++) {
        bootsSymEncrypt(&x[i], (int)((av >> i) & 1), key);
        bootsSymEncrypt(&y[i], (int)((bv >> i) & 1), key);
    }
    Cipher a(bits, x), b(bits, y);
    // the first gate call of a process builds the key's device context (HIP initialisation, code
    // objects, key upload + conversion on the GPU, this thread's lane): timed on its own, then the
    // addition itself — what the reference times too, its keys being loaded before
    LweSample *w = new_gate_bootstrapping_ciphertext_array(1, params);
    double t0 = omp_get_wtime();
    tfhe_amd_tier1_prepare(Cipher::bk);   // the context set-up, timed apart
    double tp = omp_get_wtime();
    bootsAND(w, &x[0], &y[0], Cipher::bk);
    double t1 = omp_get_wtime();
    Cipher sum = a + b;
    double t2 = omp_get_wtime();
    printf("{\"a\": %ld, \"b\": %ld, \"sum\": %ld, \"seconds\": %.4f, \"prepare_seconds\": %.4f, "
           "\"first_gate_seconds\": %.4f, \"gates\": 160, \"ms_per_gate\": %.3f}\n", decode(a, key), decode(b, key),
           decode(sum, key), t2 - t1, tp - t0, t1 - tp, 1e3 * (t2 - t1) / 160);
    delete_gate_bootstrapping_ciphertext_array(1, w);
    return 0;
}

// `cipher_ops mul16 A B [threads]`: the unchanged Cipher::operator* (Cipher.cpp:83-112) on 16-bit
// operands -> 32-bit product.  Built twice (oracle/build_callers.sh): cipher_ops runs the loop
// sequentially (Cipher.cpp leaves PARALLEL undefined), cipher_ops_par compiles Cipher.cpp with
// -DPARALLEL, so the partial products run on an OpenMP team of Cipher::nThreads = `threads`
// threads with the Cipher-sum reduction; their concurrent single-gate calls are what the
// library's Tier-1 coalescing queue batches.
static int mul16(const TFheGateBootstrappingSecretKeySet *key, long av, long bv, int threads) {
    const TFheGateBootstrappingParameterSet *params = Cipher::bk->params;
    const int bits = 16;
    LweSample *x = new_gate_bootstrapping_ciphertext_array(bits, params);
    LweSample *y = new_gate_bootstrapping_ciphertext_array(bits, params);
    for (int i = 0; i < bits; i++) {
        bootsSymEncrypt(&x[i], (int)((av >> i) & 1), key);
        bootsSymEncrypt(&y[i], (int)((bv >> i) & 1), key);
    }
    Cipher a(bits, x), b(bits, y);
    Cipher::nThreads = threads;
    LweSample *w = new_gate_bootstrapping_ciphertext_array(1, params);
    bootsAND(w, &x[0], &y[0], Cipher::bk);   // device context built outside the timed region
    long long nb0 = 0, ng0 = 0, big = 0;
    tfhe_amd_tier1_queue_stats(Cipher::bk, nullptr, nullptr, nullptr, 1);
    double t0 = omp_get_wtime();
    Cipher prod = a * b;
    double t1 = omp_get_wtime();
    tfhe_amd_tier1_queue_stats(Cipher::bk, &nb0, &ng0, &big, 0);
    printf("{\"a\": %ld, \"b\": %ld, \"prod\": %ld, \"seconds\": %.4f, \"threads\": %d, \"gates\": %lld, "
           "\"batches\": %lld, \"largest_batch\": %lld}\n", decode(a, key), decode(b, key), decode(prod, key),
           t1 - t0, threads, ng0, nb0, big);
    delete_gate_bootstrapping_ciphertext_array(1, w);
    return 0;
}

int main(int argc, char **argv) {
    FILE *f = fopen("secret.key", "rb");
    if (!f) { fprintf(stderr, "secret.key missing\n"); return 2; }
    TFheGateBootstrappingSecretKeySet *key = new_tfheGateBootstrappingSecretKeySet_fromFile(f);
    fclose(f);
    if (argc == 4 && std::string(argv[1]) == "add32") return add32(key, atol(argv[2]), atol(argv[3]));
    if (argc >= 4 && std::string(argv[1]) == "mul16")
        return mul16(key, atol(argv[2]), atol(argv[3]), argc > 4 ? atoi(argv[4]) : 4);
    const TFheGateBootstrappingParameterSet *params = Cipher::bk->params;
    const int bits = 16;
    LweSample *x = new_gate_bootstrapping_ciphertext_array(bits, params);
    LweSample *y = new_gate_bootstrapping_ciphertext_array(bits, params);
    f = fopen("cloud.data", "rb");
    if (!f) { fprintf(stderr, "cloud.data missing\n"); return 2; }
    for (int i = 0; i < bits; i++) import_gate_bootstrapping_ciphertext_fromFile(f, &x[i], params);
    for (int i = 0; i < bits; i++) import_gate_bootstrapping_ciphertext_fromFile(f, &y[i], params);
    fclose(f);

    Cipher a(bits, x), b(bits, y);
    double t0 = omp_get_wtime();
    Cipher sum = a + b;
    Cipher diff = a - b;
    Cipher lo_a(8, x), lo_b(8, y);
    Cipher prod = lo_a * lo_b;                 // 16-bit product of the low bytes
    Cipher mn = minimum(a, b);
    Cipher eq = a == b;
    Cipher gt = a > b;
    double t1 = omp_get_wtime();
    printf("{\"a\": %ld, \"b\": %ld, \"sum\": %ld, \"diff\": %ld, \"prod\": %ld, \"min\": %ld, "
           "\"eq\": %ld, \"gt\": %ld, \"seconds\": %.3f}\n",
           decode(a, key), decode(b, key), decode(sum, key), decode(diff, key), decode(prod, key),
           decode(mn, key), decode(eq, key), decode(gt, key), t1 - t0);
    return 0;
}
