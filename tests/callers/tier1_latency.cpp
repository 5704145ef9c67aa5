// tier1_latency.cpp — single-gate latency of the Tier-1 C API (what an unchanged Cipher.cpp /
// cloud.cpp caller sees per bootsNAND), built against include/ + libtfhe_amd only.  Times R
// sequential bootsNAND calls after a warm-up and prints one JSON line.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include "tfhe/tfhe.h"

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 50;
    const int seed[] = {314, 1592, 657};
    tfhe_random_generator_setSeed((uint32_t *)seed, 3);
    TFheGateBootstrappingParameterSet *params = new_default_gate_bootstrapping_parameters(110);
    TFheGateBootstrappingSecretKeySet *key = new_random_gate_bootstrapping_secret_keyset(params);
    const TFheGateBootstrappingCloudKeySet *bk = &key->cloud;
    LweSample *x = new_gate_bootstrapping_ciphertext_array(3, params);
    bootsSymEncrypt(&x[0], 1, key);
    bootsSymEncrypt(&x[1], 1, key);
    for (int i = 0; i < 3; ++i) bootsNAND(&x[2], &x[0], &x[1], bk);   // warm-up: key upload, lane
    int ok = 1;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) {
        bootsNAND(&x[2], &x[0], &x[1], bk);
        bootsNAND(&x[0], &x[2], &x[1], bk);   // x0 = NAND(NAND(x0, 1), 1) = x0: chained like a circuit
    }
    const auto t1 = std::chrono::steady_clock::now();
    ok = bootsSymDecrypt(&x[0], key) == 1 && bootsSymDecrypt(&x[2], key) == 0;
    const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count() / (2.0 * reps);
    printf("{\"tier1_ms_per_gate\": %.4f, \"gates\": %d, \"decrypt_ok\": %s}\n", ms, 2 * reps, ok ? "true" : "false");
    delete_gate_bootstrapping_ciphertext_array(3, x);
    delete_gate_bootstrapping_secret_keyset(key);
    delete_gate_bootstrapping_parameters(params);
    return ok ? 0 : 1;
}
