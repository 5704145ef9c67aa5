// param_dump.cpp — prints, as one JSON line, the gadget-decomposition constants of the default
// parameter set (TGswParams: h[], offset, kpl, Bg, halfBg, maskMod) and the index map of the
// key-switching key (the row of ks0_raw that ks[i][j][h] addresses) exactly as libtfhe_amd
// exposes them through the public TFHE structs (include/tfhe/tfhe.h), for comparison with the
// reference's own tgsw.cu / lwekeyswitch.cu (tests/golden: tgsw_*, ksk_index).  Host only.
#include <cstdio>
#include <cstdint>
#include "tfhe/tfhe.h"

int main() {
    TFheGateBootstrappingParameterSet *params = new_default_gate_bootstrapping_parameters(110);
    const TGswParams *g = params->tgsw_params;
    printf("{\"h\": [");
    for (int i = 0; i < g->l; i++) printf("%s%d", i ? ", " : "", g->h[i]);
    printf("], \"offset\": %u, \"kpl\": %d, \"Bg\": %d, \"halfBg\": %d, \"maskMod\": %u, ", g->offset, g->kpl, g->Bg,
           g->halfBg, g->maskMod);
    uint32_t seed[] = {1, 2, 3};
    tfhe_random_generator_setSeed(seed, 3);
    TFheGateBootstrappingSecretKeySet *key = new_random_gate_bootstrapping_secret_keyset(params);
    const LweKeySwitchKey *ks = key->cloud.bkFFT->ks;
    printf("\"ks_n\": %d, \"ks_t\": %d, \"ks_base\": %d, \"ksk_index\": [", ks->n, ks->t, ks->base);
    for (int i = 0; i < ks->n; i++)
        for (int j = 0; j < ks->t; j++)
            for (int h = 0; h < ks->base; h++)
                printf("%s%ld", (i | j | h) ? ", " : "", (long)(ks->ks[i][j] + h - ks->ks0_raw));
    printf("]}\n");
    delete_gate_bootstrapping_secret_keyset(key);
    delete_gate_bootstrapping_parameters(params);
    return 0;
}
