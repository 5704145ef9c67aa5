// engine.h — internal device-engine interface (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "params.h"
#include "ntt_tables.h"

namespace tfhe_amd {

// Key material of one cloud key resident on one GPU.
struct DeviceKey {
    int device = -1;
    uint32_t *bk_ntt = nullptr;   // v1: [kn][2 primes][kKpl][2][kN], Montgomery form, 1/N folded
    uint32_t *bk_v2 = nullptr;    // v2: [kn][2 primes][2 c][kKpl][4 v][64 L][4 e] (same values)
    uint2 *tw2 = nullptr;         // v2 twiddles: uniform fwd/inv [2][16] x2, streams [2][27][64], [2][18][64]
    uint2 *tw4 = nullptr;         // v4 inverse-CT twiddles: uniform [2][16], streams [2][27][64], post-twist [2][16][64]
    double2 *bk_fft = nullptr;    // v6: [kn][4 rows][2 c][8 r][64 L] FFT-domain key / 512 (slot 8 L + r)
    double2 *tw6 = nullptr;       // v6 twiddles: forward [4] + [4][64] x 2, inverse [4][64] x 2, post-twist [8][64]
    int32_t *ksk = nullptr;       // [kN][kKsT][3][kKsRow]   (digits h = 1..3)
    int32_t *ksk4 = nullptr;      // ks-v4: [126 column blocks][kN][kKsT][3][4]
    int32_t *ksk5 = nullptr;      // ks-v5 (int8 MFMA): [64 N-blocks][kN][64 lanes][16 B] signed key bytes
    NttTables *tables = nullptr;  // device copy
    uint32_t qinv_neg[2] = {0, 0};
    uint32_t crt_h = 0, crt_hp = 0;
    bool has_bk = false;
};
constexpr int kTw2Words = 2 * 16 * 2 + 2 * 27 * 64 + 2 * 18 * 64;   // uint2 entries
constexpr int kTw4Words = 2 * 16 + 2 * 27 * 64 + 2 * 16 * 64;
// double2 entries (blind_rotate_v6.hip build_v6_twiddles)
constexpr int kTw6Words = 4 + 4 * 4 * 64 + 8 * 64 + 2 * 64;   // fft_wave.h table map

// x = (0, c) + sa * X + sb * Y   (gate prologue, boot-gates.cu:98-397; Y unused if sb == 0)
struct BrInput {
    const int32_t *x_a, *x_b;
    const int32_t *y_a, *y_b;
    int32_t c, sa, sb;
};

// One bootstrapped row of a circuit level (circuit.cpp): the blind rotation input is
// (0, c) + sa W[x] + sb W[y] + sc W[z] over wire indices (-1 = absent; x is always present).
struct CircRow {
    int32_t c, sa, sb, sc;
    int32_t x, y, z, pad;
};
// One key-switched circuit output: W[out] = KS(u[r1] (+ u[r2] if r2 >= 0) + (0, add_b)).
struct CircKs {
    int32_t r1, r2, add_b, out;
};
// One bootstrap-free node: W[out] = (0, c) + s W[in]   (in = -1: the trivial sample (0, c)).
struct CircLin {
    int32_t c, s, in, out;
};

// Makes `device` current for the scope of an entry point and gives the caller's current device
// back at its end: a caller that works on another GPU (torch.cuda.set_device(1), then a
// context on device 0) keeps its own current device, which HIP and torch allocate on.
struct DeviceScope {
    int prev = -1;
    hipError_t rc;
    explicit DeviceScope(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        rc = device >= 0 && device != prev ? hipSetDevice(device) : hipSuccess;
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope &) = delete;
    DeviceScope &operator=(const DeviceScope &) = delete;
};

// Orders the reuse of a scratch buffer across streams.  Device-API callers may pass a different
// stream per call; a call on another stream than the previous user's waits (on the device) for
// the event recorded after that user's last launch, so two batches in flight never share the
// extracted samples u_a / u_b.
struct StreamFence {
    hipEvent_t ev = nullptr;
    hipStream_t last = nullptr;   // compared only; the event carries the ordering
    hipError_t acquire(hipStream_t s) const {
        return ev && last != s ? hipStreamWaitEvent(s, ev, 0) : hipSuccess;
    }
    hipError_t done(hipStream_t s) {
        if (!ev) {
            const hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        last = s;
        return hipEventRecord(ev, s);
    }
    void release() {
        if (ev) (void)hipEventDestroy(ev);
        ev = nullptr;
        last = nullptr;
    }
};

// Exactness guard of the fp64 FFT blind rotation.  The v6 kernel rounds each
// external-product coefficient c to the nearest integer; that equals the exact product while the
// FFT error stays below 1/2.  Every wave tracks the largest rounding distance |c - rint(c)| it
// sees over all 500 steps and stores its high word (monotone in the distance) in flags[2 slot + w];
// an exact-NTT (v4) launch in guard mode then recomputes every ciphertext whose flag reaches the
// threshold (1/8 by default) and exits at once for all others.  stats[0] counts the recomputed
// ciphertexts, stats[1] holds the largest high word seen (tfhe_amd_guard_stats).
struct Guard {
    uint32_t *flags = nullptr;
    uint32_t *stats = nullptr;
};
uint32_t guard_threshold_hi();

// BK conversion (coefficient -> NTT domain) on the device; d_bk_coef = [kn][4][2][kN]
hipError_t launch_bk_to_ntt(const int32_t *d_bk_coef, uint32_t *d_bk_ntt, const NttTables *d_tab,
                            hipStream_t s);
// Blind rotation + sample extraction for `halves` x B ciphertexts: ciphertext g of half h
// reads in[h] at index g and writes u[h*B + g] (u_a row stride kN).
// the NTT-domain key layouts and their twiddle streams (ntt_key.hip), used by the v4 kernels
void build_v2_twiddles(const NttTables &t, uint2 *tu_f, uint2 *tu_i, uint2 *ts_f, uint2 *ts_i);
hipError_t launch_bk_v1_to_v2(const uint32_t *d_v1, uint32_t *d_v2, hipStream_t s);
// v4 (v2 layout, inverse CT + lazy CRT + periodic accumulator), blind_rotate_v4.hip
void build_v4_twiddles(const NttTables &t, uint2 *tu_i, uint2 *ts_i, uint2 *tpost);
// guard != null: guard mode (recompute only the ciphertexts whose v6 flag reached the threshold)
hipError_t launch_blind_rotate_v4(const DeviceKey &key, int B, int halves, const BrInput *in, int32_t mu,
                                  int32_t *u_a, int32_t *u_b, hipStream_t s, const Guard *guard = nullptr);
hipError_t launch_blind_rotate_v4_debug(const DeviceKey &key, int B, int iters, int32_t *acc,
                                        const int32_t *bara, hipStream_t s);
// tGswFFTExternMulToTLwe, exact (v4 arithmetic): acc [B][2][kN] <- BK_{key_index[b]} (x) acc
hipError_t launch_external_product_v4(const DeviceKey &key, int B, const int32_t *key_index, int32_t *acc,
                                      hipStream_t s);
// circuit level (v4 kernel): B instances x nrows rows, wires [W][B] ciphertexts, u slots r B + k
hipError_t launch_blind_rotate_v4_rows(const DeviceKey &key, int B, int nrows, const CircRow *rows, const int32_t *wa,
                                       const int32_t *wb, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t s,
                                       const Guard *guard = nullptr);
// v6 (fp64 FFT external product, the reference's arithmetic), blind_rotate_v6.hip
void build_v6_twiddles(double2 *tw);
hipError_t launch_bk_to_fft(const int32_t *d_bk_coef, double2 *d_bkf, const double2 *d_tw, hipStream_t s);
// guard != null: write the rounding-distance flags (Guard) for the guard launch that follows
hipError_t launch_blind_rotate_v6(const DeviceKey &key, int B, int halves, const BrInput *in, int32_t mu,
                                  int32_t *u_a, int32_t *u_b, hipStream_t s, const Guard *guard = nullptr);
hipError_t launch_blind_rotate_v6_rows(const DeviceKey &key, int B, int nrows, const CircRow *rows, const int32_t *wa,
                                       const int32_t *wb, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t s,
                                       const Guard *guard = nullptr);
hipError_t launch_blind_rotate_v6_debug(const DeviceKey &key, int B, int iters, int32_t *acc,
                                        const int32_t *bara, hipStream_t s);
// which blind-rotation kernel runs: 0 = default (v6), 4 = exact NTT (tfhe_amd_select_kernel)
int br_version();
// Launch trace: every launcher names the kernel (and variant) it enqueues; a batch entry point of
// the C ABI collects the names of its launches into its context (tfhe_amd_last_kernels), so a
// smoke or bench run can say which kernels produced the results it checked.
void trace_kernel(const char *name);
// circuit level blind rotation with the selected kernel (rows variants of v4 / v5 / v6); the
// default fp64 kernel runs guarded (flags: 2 words per row x instance)
hipError_t launch_blind_rotate_rows(const DeviceKey &key, int B, int nrows, const CircRow *rows, const int32_t *wa,
                                    const int32_t *wb, int32_t mu, int32_t *u_a, int32_t *u_b, hipStream_t s,
                                    const Guard *guard);

// which key-switch kernel runs: 1..4 (env TFHE_AMD_KS)
int ks_version();
size_t ksk_v4_words();
size_t ksk_v5_words();
bool ks5_enabled();   // env TFHE_AMD_KS5=0: ks-v4 instead of the int8 MFMA key switch
hipError_t launch_ksk_to_v5(const int32_t *d_ksk, int32_t *d_ksk5, hipStream_t s);
// circuit level key switch: nks outputs x B instances; lane t = g B + k
hipError_t launch_keyswitch_rows(const DeviceKey &key, int B, int nks, const CircKs *ks, const int32_t *u_a,
                                 const int32_t *u_b, int32_t *wa, int32_t *wb, hipStream_t s);
// bootstrap-free nodes: nlin x B instances
hipError_t launch_circuit_linear(int B, int nlin, const CircLin *lin, int32_t *wa, int32_t *wb, hipStream_t s);
hipError_t launch_ksk_to_v4(const int32_t *d_ksk, int32_t *d_ksk4, hipStream_t s);
// current_variance of B key-switched samples u (halves = 2: u1 + u2) from the key-switching key's
// row variances var [kN][kKsT][kKsBase] (reference order of the double adds), into out [B]
hipError_t launch_ks_variance(const int32_t *u_a, int B, int halves, const double *var, double *out, hipStream_t s);
hipError_t launch_ks_variance_rows(const int32_t *u_a, int B, const CircKs *ks, const double *var, double *out,
                                   hipStream_t s);
// Key switch of u (+ u2 if non-null) + (0, add_b) -> res (n=500).
hipError_t launch_keyswitch(const DeviceKey &key, int B, const int32_t *u_a, const int32_t *u_b,
                            const int32_t *u2_a, const int32_t *u2_b, int32_t add_b,
                            int32_t *res_a, int32_t *res_b, hipStream_t s);

}  // namespace tfhe_amd
