// test_v2_parts.hip — GPU self-test of the v2 blind-rotation building blocks in isolation
// (forward / inverse register NTT against a host reference).  Debug tool, not the product.
//   hipcc -O3 -std=c++17 -fno-strict-aliasing --offload-arch=gfx950 -I cpu-gpu-tfhe_amd/csrc \
//         scripts/test_v2_parts.hip cpu-gpu-tfhe_amd/csrc/engine.cpp -o scripts/test_v2_parts
#include "blind_rotate.hip"

#include <cstdio>
#include <random>
#include <vector>
#include <cstring>

using namespace tfhe_amd;

__global__ void k_fwd(const uint2 *tu, const uint2 *ts, uint32_t *io, int s, int np) {
    __shared__ uint32_t sc[kPadRow];
    const int L = threadIdx.x;
    const uint32_t q = s ? kQ1 : kQ0;
    uint32_t x[1][16];
    for (int r = 0; r < 16; ++r) x[0][r] = io[L + 64 * r];
    ntt_fwd<1>(x, sc, tu + 16 * s, ts + s * 27 * 64 + L, L, q);
    for (int r = 0; r < 16; ++r) io[16 * L + r] = x[0][r] % q;
}

__global__ void k_inv(const uint2 *tu, const uint2 *ts, uint32_t *io, int s) {
    __shared__ uint32_t sc[kPadRow];
    const int L = threadIdx.x;
    const uint32_t q = s ? kQ1 : kQ0;
    uint32_t x[1][16];
    for (int r = 0; r < 16; ++r) x[0][r] = io[16 * L + r];
    ntt_inv<1>(x, sc, tu + 16 * s, ts + s * 18 * 64 + L, L, q);
    for (int r = 0; r < 16; ++r) io[L + 64 * r] = x[0][r] % q;
}

static void ref_fwd(std::vector<uint64_t> &a, const NttTables &t, int s) {
    const uint64_t q = kQ[s];
    int tt = kN;
    for (int m = 1; m < kN; m <<= 1) {
        tt >>= 1;
        for (int i = 0; i < m; i++) {
            const uint64_t w = t.psi[s][m + i];
            for (int j = 2 * i * tt; j < 2 * i * tt + tt; j++) {
                uint64_t u = a[j], v = a[j + tt] * w % q;
                a[j] = (u + v) % q;
                a[j + tt] = (u + q - v) % q;
            }
        }
    }
}

int main_parts() {
    NttTables *ht = new NttTables;
    build_ntt_tables(ht);
    std::vector<uint2> tw(kTw2Words);
    build_v2_twiddles(*ht, tw.data(), tw.data() + 32, tw.data() + 64, tw.data() + 64 + 2 * 27 * 64);
    uint2 *dtw;
    uint32_t *dio;
    (void)hipMalloc(&dtw, sizeof(uint2) * tw.size());
    (void)hipMemcpy(dtw, tw.data(), sizeof(uint2) * tw.size(), hipMemcpyHostToDevice);
    (void)hipMalloc(&dio, 4 * kN);
    std::mt19937_64 rng(1);
    int fails = 0;
    for (int s = 0; s < 2; ++s) {
        const uint32_t q = kQ[s];
        std::vector<uint64_t> a(kN);
        std::vector<uint32_t> h(kN);
        for (int j = 0; j < kN; j++) { a[j] = rng() % q; h[j] = (uint32_t)a[j]; }
        (void)hipMemcpy(dio, h.data(), 4 * kN, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_fwd, dim3(1), dim3(64), 0, 0, dtw, dtw + 64, dio, s, 1);
        (void)hipMemcpy(h.data(), dio, 4 * kN, hipMemcpyDeviceToHost);
        std::vector<uint64_t> want = a;
        ref_fwd(want, *ht, s);
        int bad = 0;
        for (int j = 0; j < kN; j++) bad += h[j] != want[j];
        printf("prime %d forward: %d / 1024 mismatches\n", s, bad);
        fails += bad;
        // inverse of the (correct) forward output: expect N * a
        for (int j = 0; j < kN; j++) h[j] = (uint32_t)want[j];
        (void)hipMemcpy(dio, h.data(), 4 * kN, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_inv, dim3(1), dim3(64), 0, 0, dtw + 32, dtw + 64 + 2 * 27 * 64, dio, s);
        (void)hipMemcpy(h.data(), dio, 4 * kN, hipMemcpyDeviceToHost);
        bad = 0;
        for (int j = 0; j < kN; j++) bad += (uint64_t)h[j] * ht->ninv[s] % q != a[j];
        printf("prime %d inverse: %d / 1024 mismatches\n", s, bad);
        fails += bad;
    }
    printf(fails ? "FAIL\n" : "OK\n");
    return fails ? 1 : 0;
}

// ---------------------------------------------------------------- staged CMux check
// copy of cmux_v2 with dumps (wave s writes its stage values to dump[s][stage][j])
__global__ void k_cmux_dump(V2Args g, uint32_t *acc_io, int a, uint32_t *dump) {
    __shared__ V2Shared sh;
    const int tid = threadIdx.x;
    const int s = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = tid & 63;
    for (int j = tid; j < 2 * kN; j += 128) sh.acc[j >> 10][j & 1023] = acc_io[j];
    __syncthreads();
    const uint32_t q = s ? kQ1 : kQ0;
    const uint32_t q2 = 2 * q;
    uint32_t *sc = sh.scratch[s];
    uint32_t *dmp = dump + (size_t)s * 16 * kN;   // [stage-slot][kN]
    uint32_t D[4][16];
    for (int c = 0; c < 2; ++c)
        for (int r = 0; r < 16; ++r) {
            const int j = L + 64 * r;
            const int si = (j - a) & (k2N - 1);
            const uint32_t v = sh.acc[c][si & (kN - 1)];
            const uint32_t rot = (si & kN) ? 0u - v : v;
            const uint32_t t = rot - sh.acc[c][j] + kDecompOffset;
            D[2 * c][r] = ((t >> 22) & 1023u) + (q - 512u);
            D[2 * c + 1][r] = ((t >> 12) & 1023u) + (q - 512u);
        }
    for (int p = 0; p < 4; ++p)
        for (int r = 0; r < 16; ++r) dmp[p * kN + L + 64 * r] = D[p][r] % q;          // slots 0..3: digits (A)
    ntt_fwd<4>(D, sc, g.tu_f + 16 * s, g.ts_f + s * 27 * 64 + L, L, q);
    for (int p = 0; p < 4; ++p)
        for (int r = 0; r < 16; ++r) dmp[(4 + p) * kN + 16 * L + r] = D[p][r] % q;    // slots 4..7: NTT (C)
    const uint4 *bk4 = reinterpret_cast<const uint4 *>(g.bk + ((size_t)(0 * 2 + s) * 8) * kN) + L;
    const uint32_t qinv = s ? g.qinv_neg1 : g.qinv_neg0;
    uint32_t O[2][16];
    for (int v = 0; v < 4; ++v) {
        for (int e = 0; e < 4; ++e)
            for (int p = 0; p < 4; ++p) D[p][4 * v + e] = umin32(D[p][4 * v + e], D[p][4 * v + e] - q2);
        for (int c = 0; c < 2; ++c) {
            uint4 b[4];
            for (int p = 0; p < 4; ++p) b[p] = bk4[(c * 4 + p) * 256 + v * 64];
            for (int e = 0; e < 4; ++e) {
                const uint32_t b0 = e == 0 ? b[0].x : e == 1 ? b[0].y : e == 2 ? b[0].z : b[0].w;
                const uint32_t b1 = e == 0 ? b[1].x : e == 1 ? b[1].y : e == 2 ? b[1].z : b[1].w;
                const uint32_t b2 = e == 0 ? b[2].x : e == 1 ? b[2].y : e == 2 ? b[2].z : b[2].w;
                const uint32_t b3 = e == 0 ? b[3].x : e == 1 ? b[3].y : e == 2 ? b[3].z : b[3].w;
                const int r = 4 * v + e;
                const uint64_t x = (uint64_t)D[0][r] * b0 + (uint64_t)D[1][r] * b1 + (uint64_t)D[2][r] * b2 +
                                   (uint64_t)D[3][r] * b3;
                const uint32_t m = (uint32_t)x * qinv;
                const uint32_t t = (uint32_t)((x + (uint64_t)m * q) >> 32);
                O[c][r] = umin32(t, t - q2);
            }
        }
    }
    for (int c = 0; c < 2; ++c)
        for (int r = 0; r < 16; ++r) dmp[(8 + c) * kN + 16 * L + r] = O[c][r] % q;    // slots 8,9: MAC (C)
    ntt_inv<2>(O, sc, g.tu_i + 16 * s, g.ts_i + s * 18 * 64 + L, L, q);
    for (int c = 0; c < 2; ++c)
        for (int r = 0; r < 16; ++r) dmp[(10 + c) * kN + L + 64 * r] = O[c][r] % q;   // slots 10,11: inverse (A)
    for (int c = 0; c < 2; ++c)
        for (int r = 0; r < 16; ++r) O[c][r] = umin32(O[c][r], O[c][r] - q);
    for (int c = 0; c < 2; ++c)
        for (int r = 0; r < 16; ++r) dmp[(12 + c) * kN + L + 64 * r] = O[c][r];       // slots 12,13: reduced (raw)
    if (s == 0) crt_give<0>(sh, O, L);
    else crt_give<1>(sh, O, L);
    __syncthreads();
    if (s == 0) crt_take<0>(sh, O, L, g);
    else crt_take<1>(sh, O, L, g);
    __syncthreads();
    for (int j = tid; j < 2 * kN; j += 128) acc_io[j] = sh.acc[j >> 10][j & 1023];
    if (tid == 0) { dmp[14 * kN] = g.crt_h; dmp[14 * kN + 1] = g.crt_hp; }
}

struct Ctx2 { V2Args g; };

extern "C" int run_staged(const int32_t *acc_in, int a, const int32_t *bk0 /*[4][2][kN] key index 0*/,
                          uint32_t *dump /*[2][12][kN]*/) {
    NttTables *ht = new NttTables;
    build_ntt_tables(ht);
    std::vector<uint2> tw(kTw2Words);
    build_v2_twiddles(*ht, tw.data(), tw.data() + 32, tw.data() + 64, tw.data() + 64 + 2 * 27 * 64);
    DeviceKey key;
    (void)hipMalloc(&key.tw2, sizeof(uint2) * tw.size());
    (void)hipMemcpy(key.tw2, tw.data(), sizeof(uint2) * tw.size(), hipMemcpyHostToDevice);
    (void)hipMalloc(&key.tables, sizeof(NttTables));
    (void)hipMemcpy(key.tables, ht, sizeof(NttTables), hipMemcpyHostToDevice);
    const size_t coef_words = (size_t)kn * kKpl * 2 * kN;
    std::vector<int32_t> coef(coef_words, 0);
    memcpy(coef.data(), bk0, sizeof(int32_t) * kKpl * 2 * kN);
    int32_t *dcoef;
    (void)hipMalloc(&dcoef, 4 * coef_words);
    (void)hipMemcpy(dcoef, coef.data(), 4 * coef_words, hipMemcpyHostToDevice);
    (void)hipMalloc(&key.bk_ntt, 8 * coef_words);
    (void)hipMalloc(&key.bk_v2, 8 * coef_words);
    (void)launch_bk_to_ntt(dcoef, key.bk_ntt, key.tables, 0);
    (void)launch_bk_v1_to_v2(key.bk_ntt, key.bk_v2, 0);
    key.qinv_neg[0] = ht->qinv_neg[0]; key.qinv_neg[1] = ht->qinv_neg[1];
    key.crt_h = ht->crt_h; key.crt_hp = ht->crt_hp;
    V2Args g = v2_args(key);
    uint32_t *dacc, *ddump;
    (void)hipMalloc(&dacc, 8 * kN);
    (void)hipMalloc(&ddump, 4 * 2 * 16 * kN);
    (void)hipMemcpy(dacc, acc_in, 8 * kN, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_cmux_dump, dim3(1), dim3(128), 0, 0, g, dacc, a, ddump);
    (void)hipMemcpy(dump, ddump, 4 * 2 * 16 * kN, hipMemcpyDeviceToHost);
    (void)hipMemcpy((void *)(dump + 2 * 16 * kN), dacc, 8 * kN, hipMemcpyDeviceToHost);   // staged final acc
    // also the real debug kernel on the same key for the final accumulator
    int32_t *bara;
    (void)hipMalloc(&bara, 4);
    (void)hipMemcpy(bara, &a, 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dacc, acc_in, 8 * kN, hipMemcpyHostToDevice);
    (void)launch_blind_rotate_v2_debug(key, 1, 1, (int32_t *)dacc, bara, 0);
    (void)hipMemcpy((void *)acc_in, dacc, 8 * kN, hipMemcpyDeviceToHost);   // overwritten with the result
    (void)hipDeviceSynchronize();
    // host copy of the v1 NTT key for the host-side reference
    return 0;
}
