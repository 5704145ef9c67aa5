// cipher_ops.cpp — drives the reference's own Cipher class (cpuParallel/Cipher.cpp, compiled
// unchanged by oracle/build_callers.sh) on top of libtfhe_amd, from the files the reference's
// cpuParallel/main.cpp writes (secret.key, cloud.key, cloud.data in the working directory).
// Cipher's static initialiser (Cipher.cpp:10-17) loads cloud.key before main runs.
//
// Prints one JSON line with the decrypted results of the reference's circuits:
//   a + b (operator+, Cipher.cpp ripple-carry with addBits), a - b (twosComplement + add),
//   a * b (operator*, shift-and-add; on the low 8 bits), minimum(a, b), a == b, a > b.
// Integration test only (tests/test_io.py::test_reference_callers_gpu).
#include <cstdio>
#include <cstdlib>
#include <omp.h>

#include "Cipher.h"

static long decode(const Cipher &c, const TFheGateBootstrappingSecretKeySet *key) {
    long v = 0;
    for (int i = 0; i < c.numberOfBits; i++) v |= (long)bootsSymDecrypt(&c.data[i], key) << i;
    return v;
}

int main() {
    FILE *f = fopen("secret.key", "rb");
    if (!f) { fprintf(stderr, "secret.key missing\n"); return 2; }
    TFheGateBootstrappingSecretKeySet *key = new_tfheGateBootstrappingSecretKeySet_fromFile(f);
    fclose(f);
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
