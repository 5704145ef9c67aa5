// tfhe_io.cpp — key / ciphertext files in the reference's byte format (include/tfhe/tfhe_io.h).
//
// Restates gpuParallel/tfhe_io.cu and the text-section codec of tfhe_generic_streams.cu so a
// cloud.key / secret.key / cloud.data written by the reference's cpuParallel/main.cpp is
// read here and vice versa.  Host-only (file I/O is not on the bootstrapping hot path); a
// cloud keyset read from disk is uploaded to the GPU lazily on its first gate, exactly like
// one made by new_random_gate_bootstrapping_secret_keyset.
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <istream>
#include <map>
#include <ostream>
#include <string>

#include "api_internal.h"
#include "../../include/tfhe/tfhe_io.h"

using namespace tfhe_amd;
using namespace tfhe_amd::api;

namespace {

// type uids, gpuParallel/tfhe_generic_streams.h:15-30
constexpr int32_t kUidLweSample = 42;
constexpr int32_t kUidLweKey = 43;
constexpr int32_t kUidTGswKey = 169;
constexpr int32_t kUidKeySwitchKey = 200;
constexpr int32_t kUidBootstrappingKey = 201;

// ---------------------------------------------------------------- byte sinks / sources
// (the reference's Ostream/Istream pair, tfhe_generic_streams.cu:62-110)

struct Sink {
    virtual void text(const std::string &s) = 0;
    virtual void bytes(const void *p, size_t n) = 0;
    virtual ~Sink() = default;
};
struct FileSink final : Sink {
    FILE *f;
    explicit FileSink(FILE *f_) : f(f_) {}
    void text(const std::string &s) override { bytes(s.data(), s.size()); }
    void bytes(const void *p, size_t n) override {
        if (n && std::fwrite(p, 1, n, f) != n) die_dramatically("tfhe_io: short write");
    }
};
struct StreamSink final : Sink {
    std::ostream &o;
    explicit StreamSink(std::ostream &o_) : o(o_) {}
    void text(const std::string &s) override { o << s; }
    void bytes(const void *p, size_t n) override { o.write(static_cast<const char *>(p), (std::streamsize)n); }
};

struct Source {
    // one line without its '\n'; false once the end of input was hit while reading it
    // (the reference's getLine + feof pair: a last line without '\n' is dropped)
    virtual bool line(std::string &out) = 0;
    virtual void bytes(void *p, size_t n) = 0;
    virtual ~Source() = default;
};
struct FileSource final : Source {
    FILE *f;
    explicit FileSource(FILE *f_) : f(f_) {}
    bool line(std::string &out) override {
        out.clear();
        for (int c = std::fgetc(f); c != EOF; c = std::fgetc(f)) {
            if (c == '\r') continue;             // CIstream::getLine skips CR
            if (c == '\n') return true;
            out.push_back((char)c);
        }
        return false;
    }
    void bytes(void *p, size_t n) override {
        if (n && std::fread(p, 1, n, f) != n) die_dramatically("tfhe_io: unexpected end of file");
    }
};
struct StreamSource final : Source {
    std::istream &in;
    explicit StreamSource(std::istream &in_) : in(in_) {}
    bool line(std::string &out) override { return (bool)std::getline(in, out); }
    void bytes(void *p, size_t n) override {
        in.read(static_cast<char *>(p), (std::streamsize)n);
        if ((size_t)in.gcount() != n) die_dramatically("tfhe_io: unexpected end of stream");
    }
};

template <class T>
void put(Sink &s, const T &v) { s.bytes(&v, sizeof(T)); }
template <class T>
T get(Source &s) {
    T v;
    s.bytes(&v, sizeof(T));
    return v;
}

// ---------------------------------------------------------------- text sections
// tfhe_generic_streams.cu:122-186: a std::map (so names come out sorted), "%ld" / "%.8lf"

struct Section {
    std::string title;
    std::map<std::string, std::string> kv;

    void set_long(const char *k, long v) {
        char buf[64];
        snprintf(buf, sizeof buf, "%ld", v);
        kv[k] = buf;
    }
    void set_double(const char *k, double v) {
        char buf[512];                            // "%.8lf" of any double fits
        snprintf(buf, sizeof buf, "%.8lf", v);
        kv[k] = buf;
    }
    const std::string &raw(const char *k) const {
        auto it = kv.find(k);
        if (it == kv.end()) die_dramatically((std::string("tfhe_io: missing property ") + k + " in " + title).c_str());
        return it->second;
    }
    long get_long(const char *k) const {           // stol
        const std::string &v = raw(k);
        char *end = nullptr;
        errno = 0;
        long r = strtol(v.c_str(), &end, 10);
        if (end == v.c_str() || errno) die_dramatically("tfhe_io: bad integer property");
        return r;
    }
    double get_double(const char *k) const {       // stold
        const std::string &v = raw(k);
        char *end = nullptr;
        long double r = strtold(v.c_str(), &end);
        if (end == v.c_str()) die_dramatically("tfhe_io: bad real property");
        return (double)r;
    }
    void write(Sink &s) const {
        s.text("-----BEGIN " + title + "-----\n");
        for (const auto &e : kv) s.text(e.first + ": " + e.second + "\n");
        s.text("-----END " + title + "-----\n");
    }
};

// new_TextModeProperties_fromIstream: lines before BEGIN and lines without ": " are ignored;
// the section ends at its own END line.  Aborts (the reference returns NULL and crashes on
// it) when the input ends first, and when the title is not the one expected.
Section read_section(Source &src, const char *expect) {
    Section sec;
    std::string line, end_line;
    bool started = false;
    while (src.line(line)) {
        const size_t n = line.size();
        if (n >= 16 && line.compare(0, 11, "-----BEGIN ") == 0 && line.compare(n - 5, 5, "-----") == 0) {
            sec.title = line.substr(11, n - 16);
            end_line = "-----END " + sec.title + "-----";
            started = true;
            continue;
        }
        if (!started) continue;
        if (line == end_line) {
            if (sec.title != expect)
                die_dramatically((std::string("tfhe_io: expected section ") + expect + ", found " + sec.title).c_str());
            return sec;
        }
        const size_t pos = line.find(": ");
        if (pos == std::string::npos) continue;
        sec.kv[line.substr(0, pos)] = line.substr(pos + 2);
    }
    die_dramatically((std::string("tfhe_io: end of input before section ") + expect).c_str());
    return sec;
}

// ---------------------------------------------------------------- parameter sets
// write_tfheGateBootstrappingParameters (tfhe_io.cu:1014-1035): GATEBOOTSPARAMS,
// LWEPARAMS (:33-43), TLWEPARAMS (:243-253), TGSWPARAMS (:480-495)

void write_params(Sink &s, const TFheGateBootstrappingParameterSet *p) {
    Section g{"GATEBOOTSPARAMS", {}};
    g.set_long("ks_t", p->ks_t);
    g.set_long("ks_basebit", p->ks_basebit);
    g.write(s);
    const LweParams *lw = p->in_out_params;
    Section l{"LWEPARAMS", {}};
    l.set_long("n", lw->n);
    l.set_double("alpha_min", lw->alpha_min);
    l.set_double("alpha_max", lw->alpha_max);
    l.write(s);
    const TLweParams *tl = p->tgsw_params->tlwe_params;
    Section t{"TLWEPARAMS", {}};
    t.set_long("N", tl->N);
    t.set_long("k", tl->k);
    t.set_double("alpha_min", tl->alpha_min);
    t.set_double("alpha_max", tl->alpha_max);
    t.write(s);
    Section gs{"TGSWPARAMS", {}};
    gs.set_long("l", p->tgsw_params->l);
    gs.set_long("Bgbit", p->tgsw_params->Bgbit);
    gs.write(s);
}

// read_new_tfheGateBootstrappingParameters (tfhe_io.cu:1037-1047).  The engine's kernels
// are compiled for the default shape, so any other shape is refused here, loudly.
const ParamsImpl *read_params(Source &src) {
    const Section g = read_section(src, "GATEBOOTSPARAMS");
    const long ks_t = g.get_long("ks_t");
    const long ks_basebit = (long)g.get_double("ks_basebit");   // read as a double (:1026)
    const Section l = read_section(src, "LWEPARAMS");
    const Section t = read_section(src, "TLWEPARAMS");
    const Section gs = read_section(src, "TGSWPARAMS");
    if (ks_t != kKsT || ks_basebit != kKsBasebit || l.get_long("n") != kn || t.get_long("N") != kN ||
        t.get_long("k") != kK || gs.get_long("l") != kL || gs.get_long("Bgbit") != kBgbit)
        die_dramatically("tfhe_io: parameter set is not the default 128-bit gate-bootstrapping set "
                         "(n=500 N=1024 k=1 l=2 Bgbit=10 ks_t=8 ks_basebit=2) this engine is built for");
    ParamsImpl *p = new ParamsImpl(l.get_double("alpha_min"), l.get_double("alpha_max"),
                                   t.get_double("alpha_min"), t.get_double("alpha_max"));
    register_params(p);
    return p;
}

// ---------------------------------------------------------------- samples and keys

// write_lweSample / read_lweSample (tfhe_io.cu:90-110)
void write_lwe_sample(Sink &s, const LweSample *x, int n) {
    put(s, kUidLweSample);
    s.bytes(x->a, sizeof(Torus32) * (size_t)n);
    put(s, x->b);
    put(s, x->current_variance);
}
void read_lwe_sample(Source &src, LweSample *x, int n) {
    if (get<int32_t>(src) != kUidLweSample) die_dramatically("tfhe_io: not an LWE sample");
    src.bytes(x->a, sizeof(Torus32) * (size_t)n);
    x->b = get<Torus32>(src);
    x->current_variance = get<double>(src);
}

// write_lweBootstrappingKey(F, bk, false, false) (tfhe_io.cu:937-945): LWEKSPARAMS (:731-739),
// KSK content (:757-788), BK content (:883-909)
void write_bootstrapping_key(Sink &s, const LweBootstrappingKey *bk) {
    const LweKeySwitchKey *ks = bk->ks;
    Section kp{"LWEKSPARAMS", {}};
    kp.set_long("n", ks->n);
    kp.set_long("t", ks->t);
    kp.set_long("basebit", ks->basebit);
    kp.write(s);

    const int n_out = ks->out_params->n;
    double var = -1;
    for (int i = 0; i < ks->n; i++)
        for (int j = 0; j < ks->t; j++)
            for (int h = 0; h < ks->base; h++)
                if (ks->ks[i][j][h].current_variance > var) var = ks->ks[i][j][h].current_variance;
    put(s, kUidKeySwitchKey);
    put(s, var);
    for (int i = 0; i < ks->n; i++)
        for (int j = 0; j < ks->t; j++)
            for (int h = 0; h < ks->base; h++) {
                const LweSample &x = ks->ks[i][j][h];
                s.bytes(x.a, sizeof(Torus32) * (size_t)n_out);
                put(s, x.b);
            }

    const int n = bk->in_out_params->n, kpl = bk->bk_params->kpl;
    const int k = bk->bk_params->tlwe_params->k, N = bk->bk_params->tlwe_params->N;
    var = -1;
    for (int i = 0; i < n; i++)
        for (int p = 0; p < kpl; p++)
            if (bk->bk[i].all_sample[p].current_variance > var) var = bk->bk[i].all_sample[p].current_variance;
    put(s, kUidBootstrappingKey);
    put(s, var);
    for (int i = 0; i < n; i++)
        for (int p = 0; p < kpl; p++)
            for (int c = 0; c <= k; c++) s.bytes(bk->bk[i].all_sample[p].a[c].coefsT, sizeof(Torus32) * (size_t)N);
}

// read_new_lweBootstrappingKey with known params (tfhe_io.cu:951-973)
LweBootstrappingKey *read_bootstrapping_key(Source &src, const ParamsImpl *P) {
    const Section kp = read_section(src, "LWEKSPARAMS");
    if (kp.get_long("n") != (long)kN * kK) die_dramatically("Wrong dimension in bootstrapping key");
    if (kp.get_long("t") != kKsT || kp.get_long("basebit") != kKsBasebit)
        die_dramatically("tfhe_io: key-switching key shape differs from the default t=8 basebit=2");
    LweBootstrappingKey *bk = new_bk(P);

    LweKeySwitchKey *ks = bk->ks;
    if (get<int32_t>(src) != kUidKeySwitchKey) die_dramatically("Trying to read something that is not a LWE Keyswitch!");
    double var = get<double>(src);
    for (int i = 0; i < ks->n; i++)
        for (int j = 0; j < ks->t; j++)
            for (int h = 0; h < ks->base; h++) {
                LweSample &x = ks->ks[i][j][h];
                src.bytes(x.a, sizeof(Torus32) * (size_t)kn);
                x.b = get<Torus32>(src);
                x.current_variance = var;
            }

    if (get<int32_t>(src) != kUidBootstrappingKey) die_dramatically("Trying to read something that is not a BK content");
    var = get<double>(src);
    for (int i = 0; i < kn; i++)
        for (int p = 0; p < kKpl; p++) {
            TLweSample &row = bk->bk[i].all_sample[p];
            for (int c = 0; c <= kK; c++) src.bytes(row.a[c].coefsT, sizeof(Torus32) * (size_t)kN);
            row.current_variance = var;
        }
    return bk;
}

// ---------------------------------------------------------------- keysets
// write_tfheGateBootstrappingCloudKeySet (tfhe_io.cu:1099-1103) /
// read_new_tfheGateBootstrappingCloudKeySet (:1087-1097)

void write_cloud(Sink &s, const TFheGateBootstrappingCloudKeySet *key) {
    write_params(s, key->params);
    write_bootstrapping_key(s, key->bk);
}

TFheGateBootstrappingCloudKeySet *read_cloud(Source &src) {
    const ParamsImpl *P = read_params(src);
    LweBootstrappingKey *bk = read_bootstrapping_key(src, P);
    LweBootstrappingKeyFFT *bkfft = new_bkfft(bk);      // new_LweBootstrappingKeyFFT(bk), :1095
    return new TFheGateBootstrappingCloudKeySet{&P->set, bk, bkfft};
}

// write_tfheGateBootstrappingSecretKeySet (tfhe_io.cu:1160-1166): cloud part, then
// write_lweKey(F, key, false) (:168-172, :197) and write_tGswKey(F, key, false) (:660-668)
void write_secret(Sink &s, const TFheGateBootstrappingSecretKeySet *key) {
    write_params(s, key->params);
    write_bootstrapping_key(s, key->cloud.bk);
    put(s, kUidLweKey);
    s.bytes(key->lwe_key->key, sizeof(int) * (size_t)key->lwe_key->params->n);
    put(s, kUidTGswKey);
    const TLweParams *tl = key->tgsw_key->params->tlwe_params;
    for (int i = 0; i < tl->k; i++) s.bytes(key->tgsw_key->key[i].coefs, sizeof(int) * (size_t)tl->N);
}

// read_new_tfheGateBootstrappingSecretKeySet (tfhe_io.cu:1146-1158)
TFheGateBootstrappingSecretKeySet *read_secret(Source &src) {
    const ParamsImpl *P = read_params(src);
    LweBootstrappingKey *bk = read_bootstrapping_key(src, P);
    LweKey *lwe_key = new_LweKey(&P->in_out);
    if (get<int32_t>(src) != kUidLweKey) die_dramatically("tfhe_io: not an LWE key");
    src.bytes(lwe_key->key, sizeof(int) * (size_t)kn);
    TGswKey *tgsw = new_tgsw_key(P);
    if (get<int32_t>(src) != kUidTGswKey) die_dramatically("tfhe_io: not a TGSW key");
    for (int i = 0; i < kK; i++) src.bytes(tgsw->key[i].coefs, sizeof(int) * (size_t)kN);
    LweBootstrappingKeyFFT *bkfft = new_bkfft(bk);
    return new TFheGateBootstrappingSecretKeySet{&P->set, lwe_key, tgsw,
                                                 TFheGateBootstrappingCloudKeySet{&P->set, bk, bkfft}};
}

}  // namespace

// ---------------------------------------------------------------- exported entry points

EXPORT void export_lweSample_toFile(FILE *F, const LweSample *x, const LweParams *params) {
    FileSink s(F);
    write_lwe_sample(s, x, params->n);
}
EXPORT void import_lweSample_fromFile(FILE *F, LweSample *x, const LweParams *params) {
    FileSource s(F);
    read_lwe_sample(s, x, params->n);
}
EXPORT void export_lweSample_toStream(std::ostream &F, const LweSample *x, const LweParams *params) {
    StreamSink s(F);
    write_lwe_sample(s, x, params->n);
}
EXPORT void import_lweSample_fromStream(std::istream &in, LweSample *x, const LweParams *params) {
    StreamSource s(in);
    read_lwe_sample(s, x, params->n);
}

EXPORT void export_tfheGateBootstrappingParameterSet_toFile(FILE *F, const TFheGateBootstrappingParameterSet *params) {
    FileSink s(F);
    write_params(s, params);
}
EXPORT TFheGateBootstrappingParameterSet *new_tfheGateBootstrappingParameterSet_fromFile(FILE *F) {
    FileSource s(F);
    return const_cast<TFheGateBootstrappingParameterSet *>(&read_params(s)->set);
}
EXPORT void export_tfheGateBootstrappingParameterSet_toStream(std::ostream &F,
                                                              const TFheGateBootstrappingParameterSet *params) {
    StreamSink s(F);
    write_params(s, params);
}
EXPORT TFheGateBootstrappingParameterSet *new_tfheGateBootstrappingParameterSet_fromStream(std::istream &F) {
    StreamSource s(F);
    return const_cast<TFheGateBootstrappingParameterSet *>(&read_params(s)->set);
}

EXPORT void export_tfheGateBootstrappingCloudKeySet_toFile(FILE *F, const TFheGateBootstrappingCloudKeySet *key) {
    FileSink s(F);
    write_cloud(s, key);
}
EXPORT TFheGateBootstrappingCloudKeySet *new_tfheGateBootstrappingCloudKeySet_fromFile(FILE *F) {
    FileSource s(F);
    return read_cloud(s);
}
EXPORT void export_tfheGateBootstrappingCloudKeySet_toStream(std::ostream &F, const TFheGateBootstrappingCloudKeySet *key) {
    StreamSink s(F);
    write_cloud(s, key);
}
EXPORT TFheGateBootstrappingCloudKeySet *new_tfheGateBootstrappingCloudKeySet_fromStream(std::istream &F) {
    StreamSource s(F);
    return read_cloud(s);
}

EXPORT void export_tfheGateBootstrappingSecretKeySet_toFile(FILE *F, const TFheGateBootstrappingSecretKeySet *key) {
    FileSink s(F);
    write_secret(s, key);
}
EXPORT TFheGateBootstrappingSecretKeySet *new_tfheGateBootstrappingSecretKeySet_fromFile(FILE *F) {
    FileSource s(F);
    return read_secret(s);
}
EXPORT void export_tfheGateBootstrappingSecretKeySet_toStream(std::ostream &F,
                                                              const TFheGateBootstrappingSecretKeySet *key) {
    StreamSink s(F);
    write_secret(s, key);
}
EXPORT TFheGateBootstrappingSecretKeySet *new_tfheGateBootstrappingSecretKeySet_fromStream(std::istream &F) {
    StreamSource s(F);
    return read_secret(s);
}

// export/import_gate_bootstrapping_ciphertext (tfhe_io.cu:1214-1250) = the LWE sample codec
EXPORT void export_gate_bootstrapping_ciphertext_toFile(FILE *F, const LweSample *sample,
                                                        const TFheGateBootstrappingParameterSet *params) {
    export_lweSample_toFile(F, sample, params->in_out_params);
}
EXPORT void import_gate_bootstrapping_ciphertext_fromFile(FILE *F, LweSample *sample,
                                                          const TFheGateBootstrappingParameterSet *params) {
    import_lweSample_fromFile(F, sample, params->in_out_params);
}
EXPORT void export_gate_bootstrapping_ciphertext_toStream(std::ostream &F, const LweSample *sample,
                                                          const TFheGateBootstrappingParameterSet *params) {
    export_lweSample_toStream(F, sample, params->in_out_params);
}
EXPORT void import_gate_bootstrapping_ciphertext_fromStream(std::istream &F, LweSample *sample,
                                                            const TFheGateBootstrappingParameterSet *params) {
    import_lweSample_fromStream(F, sample, params->in_out_params);
}
