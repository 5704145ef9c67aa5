// api_misc.cpp — the host-side TFHE API surface that the reference's own callers do not reach but
// a libtfhe user may (include/tfhe/tfhe.h, tfhe_io.h): the std::stream readers / writers (byte-for-
// byte the FILE* ones, and round-tripping), single-LweSample I/O, the single / array allocators,
// lweClear, lweSymEncryptWithExternalNoise, t32tod.  Built against include/ + libtfhe_amd alone;
// host only (no GPU).  Prints one JSON line: every check's name and whether it held.
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <functional>
#include <sstream>
#include <string>
#include <vector>
#include "tfhe/tfhe.h"
#include "tfhe/tfhe_io.h"

static std::string via_file(const std::function<void(FILE *)> &w) {
    FILE *f = tmpfile();
    w(f);
    fflush(f);
    std::string s;
    long len = ftell(f);
    rewind(f);
    s.resize((size_t)len);
    if (len > 0 && fread(&s[0], 1, (size_t)len, f) != (size_t)len) s.clear();
    fclose(f);
    return s;
}

static std::string via_stream(const std::function<void(std::ostream &)> &w) {
    std::ostringstream o;
    w(o);
    return o.str();
}

static std::vector<std::pair<std::string, bool>> checks;
static void check(const char *name, bool ok) { checks.emplace_back(name, ok); }

static bool same_sample(const LweSample *x, const LweSample *y, int n) {
    for (int i = 0; i < n; ++i)
        if (x->a[i] != y->a[i]) return false;
    return x->b == y->b && x->current_variance == y->current_variance;
}

int main() {
    TFheGateBootstrappingParameterSet *params = new_default_gate_bootstrapping_parameters(110);
    const LweParams *io = params->in_out_params;
    const int n = io->n;
    uint32_t seed[] = {314, 1592, 657};
    tfhe_random_generator_setSeed(seed, 3);
    TFheGateBootstrappingSecretKeySet *key = new_random_gate_bootstrapping_secret_keyset(params);

    // parameter set
    {
        std::string f = via_file([&](FILE *F) { export_tfheGateBootstrappingParameterSet_toFile(F, params); });
        std::string s = via_stream([&](std::ostream &o) { export_tfheGateBootstrappingParameterSet_toStream(o, params); });
        check("params_stream_eq_file", !f.empty() && f == s);
        std::istringstream in(s);
        TFheGateBootstrappingParameterSet *p2 = new_tfheGateBootstrappingParameterSet_fromStream(in);
        std::string s2 = via_stream([&](std::ostream &o) { export_tfheGateBootstrappingParameterSet_toStream(o, p2); });
        check("params_stream_roundtrip", s2 == s && p2->in_out_params->n == n);
        delete_gate_bootstrapping_parameters(p2);
    }
    // secret keyset (LWE key, TGSW key and the cloud keys derived from them)
    std::string cloud_bytes;
    {
        std::string f = via_file([&](FILE *F) { export_tfheGateBootstrappingSecretKeySet_toFile(F, key); });
        std::string s = via_stream([&](std::ostream &o) { export_tfheGateBootstrappingSecretKeySet_toStream(o, key); });
        check("secret_stream_eq_file", !f.empty() && f == s);
        std::istringstream in(s);
        TFheGateBootstrappingSecretKeySet *k2 = new_tfheGateBootstrappingSecretKeySet_fromStream(in);
        std::string s2 = via_stream([&](std::ostream &o) { export_tfheGateBootstrappingSecretKeySet_toStream(o, k2); });
        check("secret_stream_roundtrip", s2 == s);
        delete_gate_bootstrapping_secret_keyset(k2);
    }
    // cloud keyset
    {
        std::string f = via_file([&](FILE *F) { export_tfheGateBootstrappingCloudKeySet_toFile(F, &key->cloud); });
        std::string s = via_stream([&](std::ostream &o) { export_tfheGateBootstrappingCloudKeySet_toStream(o, &key->cloud); });
        check("cloud_stream_eq_file", !f.empty() && f == s);
        std::istringstream in(s);
        TFheGateBootstrappingCloudKeySet *c2 = new_tfheGateBootstrappingCloudKeySet_fromStream(in);
        std::string s2 = via_stream([&](std::ostream &o) { export_tfheGateBootstrappingCloudKeySet_toStream(o, c2); });
        check("cloud_stream_roundtrip", s2 == s);
        delete_gate_bootstrapping_cloud_keyset(c2);
        cloud_bytes = s;
    }
    // gate-bootstrapping ciphertexts: single allocator, stream / file writers, readers
    {
        bool eq = true, rt = true, dec = true;
        for (int m = 0; m < 16; ++m) {
            LweSample *c = new_gate_bootstrapping_ciphertext(params);
            bootsSymEncrypt(c, m & 1, key);
            std::string f = via_file([&](FILE *F) { export_gate_bootstrapping_ciphertext_toFile(F, c, params); });
            std::string s = via_stream([&](std::ostream &o) { export_gate_bootstrapping_ciphertext_toStream(o, c, params); });
            eq = eq && !f.empty() && f == s;
            LweSample *d = new_gate_bootstrapping_ciphertext(params);
            std::istringstream in(s);
            import_gate_bootstrapping_ciphertext_fromStream(in, d, params);
            rt = rt && same_sample(c, d, n);
            dec = dec && bootsSymDecrypt(d, key) == (m & 1);
            delete_gate_bootstrapping_ciphertext(d);
            delete_gate_bootstrapping_ciphertext(c);
        }
        check("ciphertext_stream_eq_file", eq);
        check("ciphertext_stream_roundtrip", rt);
        check("ciphertext_stream_decrypts", dec);
    }
    // single LweSample I/O on the in/out parameters, arrays of samples
    {
        LweSample *arr = new_LweSample_array(5, io);
        for (int k = 0; k < 5; ++k) lweSymEncrypt(&arr[k], modSwitchToTorus32(k, 8), 1e-5, key->lwe_key);
        bool eq = true, rt_file = true, rt_stream = true;
        LweSample *back = new_LweSample_array(5, io);
        for (int k = 0; k < 5; ++k) {
            std::string f = via_file([&](FILE *F) { export_lweSample_toFile(F, &arr[k], io); });
            std::string s = via_stream([&](std::ostream &o) { export_lweSample_toStream(o, &arr[k], io); });
            eq = eq && !f.empty() && f == s;
            FILE *F = tmpfile();
            export_lweSample_toFile(F, &arr[k], io);
            rewind(F);
            import_lweSample_fromFile(F, &back[k], io);
            fclose(F);
            rt_file = rt_file && same_sample(&arr[k], &back[k], n);
            lweClear(&back[k], io);
            std::istringstream in(s);
            import_lweSample_fromStream(in, &back[k], io);
            rt_stream = rt_stream && same_sample(&arr[k], &back[k], n);
        }
        check("lwesample_stream_eq_file", eq);
        check("lwesample_file_roundtrip", rt_file);
        check("lwesample_stream_roundtrip", rt_stream);
        // lweClear: the noiseless zero sample
        lweClear(&back[0], io);
        bool zero = back[0].b == 0 && back[0].current_variance == 0.0;
        for (int i = 0; i < n; ++i) zero = zero && back[0].a[i] == 0;
        check("lweClear_zero", zero);
        // lweSymEncryptWithExternalNoise: phase = message + dtot32(noise) exactly, variance alpha^2
        const Torus32 msg = modSwitchToTorus32(1, 8);
        const double noise = 0.00123, alpha = 0.0042;
        lweSymEncryptWithExternalNoise(&back[1], msg, noise, alpha, key->lwe_key);
        const Torus32 ph = lwePhase(&back[1], key->lwe_key);
        check("external_noise_phase", (uint32_t)ph == (uint32_t)msg + (uint32_t)dtot32(noise));
        check("external_noise_variance", back[1].current_variance == alpha * alpha);
        delete_LweSample_array(5, back);
        delete_LweSample_array(5, arr);
    }
    // t32tod: the inverse of dtot32 on the torus grid
    {
        bool ok = t32tod(0) == 0.0 && t32tod(1 << 30) == 0.25 && t32tod(INT32_MIN) == -0.5 &&
                  t32tod(modSwitchToTorus32(1, 8)) == 0.125 && t32tod(dtot32(0.3)) == std::ldexp((double)dtot32(0.3), -32);
        check("t32tod", ok);
    }
    delete_gate_bootstrapping_secret_keyset(key);
    delete_gate_bootstrapping_parameters(params);

    int bad = 0;
    printf("{\"checks\": {");
    for (size_t i = 0; i < checks.size(); ++i) {
        printf("%s\"%s\": %s", i ? ", " : "", checks[i].first.c_str(), checks[i].second ? "true" : "false");
        bad += !checks[i].second;
    }
    printf("}, \"failed\": %d, \"cloud_bytes\": %zu}\n", bad, cloud_bytes.size());
    return bad ? 1 : 0;
}
