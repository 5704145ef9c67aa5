// keyswitch.hip — lweKeySwitch as a coalesced gather-accumulate on gfx950.
//
// Reference path replaced (gpuParallel/):
//   lweKeySwitch                       lwe-keyswitch-functions.cu:955-987
//   lweKeySwitchTranslate_fromArray    :101-127   (aibar = a_i + 2^15; 8 base-4 digits;
//                                                  result -= ks[i][j][aij] for aij != 0)
//   key layout ks[i][j][h]             lwekeyswitch.cu:3-18 (ks[i][j][0] is a zero sample :919)
// and the reference GPU comparator keySwitch_n_Bit (boot-gates.cu:2425-2479), whose KS
// kernel did 8192 dependent gathers per thread with the b-sum and the accumulator
// round-tripped through the host.
//
// Device KSK layout: [i < 1024][j < 8][h-1 < 3][512] int32, a row = 500 a + b + pad (2 KB).
// v1: one 512-thread workgroup per ciphertext, thread k owns output coefficient k
// (k == 500 is b); every (i, j) step is one 2 KB coalesced row read.  Digits are wave-
// uniform (same (i, j) for all lanes), so the aij == 0 skip never diverges.
#include "engine.h"
#include "modarith.h"

#include <cstdlib>

namespace tfhe_amd {

namespace {

constexpr int kKsThreads = 512;

__global__ __launch_bounds__(kKsThreads) void k_keyswitch_v1(
    const int32_t *__restrict__ ksk, const int32_t *__restrict__ u_a, const int32_t *__restrict__ u_b,
    const int32_t *__restrict__ u2_a, const int32_t *__restrict__ u2_b, int32_t add_b,
    int32_t *__restrict__ res_a, int32_t *__restrict__ res_b) {
    __shared__ uint32_t aibar[kN];
    const int g = blockIdx.x;
    const int tid = threadIdx.x;
    for (int i = tid; i < kN; i += kKsThreads) {
        uint32_t a = (uint32_t)u_a[(size_t)g * kN + i];
        if (u2_a) a += (uint32_t)u2_a[(size_t)g * kN + i];
        aibar[i] = a + kKsPrecOffset;
    }
    __syncthreads();
    uint32_t acc = 0;
    if (tid == kn) {
        acc = (uint32_t)u_b[g] + (uint32_t)add_b;
        if (u2_b) acc += (uint32_t)u2_b[g];
    }
    const int32_t *col = ksk + tid;
    for (int i = 0; i < kN; ++i) {
        const uint32_t ab = aibar[i];
        const int32_t *rowi = col + (size_t)i * kKsT * 3 * kKsRow;
#pragma unroll
        for (int j = 0; j < kKsT; ++j) {
            const uint32_t aij = (ab >> (32 - (j + 1) * kKsBasebit)) & (kKsBase - 1);
            if (aij) acc -= (uint32_t)rowi[(j * 3 + (int)aij - 1) * kKsRow];
        }
    }
    if (tid < kn) res_a[(size_t)g * kn + tid] = (int32_t)acc;
    else if (tid == kn) res_b[g] = (int32_t)acc;
}

// ---------------------------------------------------------------- v2
// Workgroup = 4 waves; owns a 64-column slice (lane = column) of the output for kKsCt
// ciphertexts (kKsCt / 4 per wave).  For a chunk of kKsI key indices i it stages the row
// slices KS[i][j][h][cols] (h = 1..3) in LDS once and every wave applies them to its
// ciphertexts: the digit aij is wave-uniform (SALU), so each (i, j, ct) costs one LDS read
// and one subtract, and the KSK is read from L2 once per workgroup instead of once per
// ciphertext.  Column block = blockIdx % 8: under round-robin XCD placement every XCD
// streams one 6.3 MB slice of the 50 MB key in lockstep (speed only, never correctness).
constexpr int kKsCt = 16;
constexpr int kKsI = 8;
constexpr int kKsV2Threads = 256;

__global__ __launch_bounds__(kKsV2Threads) void k_keyswitch_v2(
    const int32_t *__restrict__ ksk, int B, const int32_t *__restrict__ u_a, const int32_t *__restrict__ u_b,
    const int32_t *__restrict__ u2_a, const int32_t *__restrict__ u2_b, int32_t add_b,
    int32_t *__restrict__ res_a, int32_t *__restrict__ res_b) {
    // rows[(ii * 8 + j) * 4 + h][col]: h = 0 is a resident zero row (the digit-0 term of
    // lwe-keyswitch-functions.cu:919), so the gather is branch-free and the LDS reads batch
    __shared__ __attribute__((aligned(16))) uint32_t rows[kKsI * kKsT * 4][64];   // 64 KB
    const int cb = blockIdx.x & 7;                  // column block: columns [64 cb, 64 cb + 64)
    const int ct0 = (blockIdx.x >> 3) * kKsCt;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int col = cb * 64 + lane;
    constexpr int kPerWave = kKsCt / 4;
    uint32_t acc[kPerWave];
#pragma unroll
    for (int k = 0; k < kPerWave; ++k) {
        const int g = ct0 + wave * kPerWave + k;
        acc[k] = 0;
        if (col == kn && g < B) acc[k] = (uint32_t)u_b[g] + (uint32_t)add_b + (u2_b ? (uint32_t)u2_b[g] : 0u);
    }
    for (int t = tid; t < kKsI * kKsT * 64; t += kKsV2Threads) rows[(t >> 6) * 4][t & 63] = 0;
    for (int i0 = 0; i0 < kN; i0 += kKsI) {
        // stage 24 kKsI rows x 64 columns (uint4 per thread-slot) into the h = 1..3 slots
        const int32_t *src = ksk + (size_t)i0 * kKsT * 3 * kKsRow + cb * 64;
        for (int t = tid; t < kKsI * kKsT * 3 * 16; t += kKsV2Threads) {
            const int row = t >> 4, c4 = (t & 15) * 4;
            const int ij = row / 3, h = row - 3 * ij + 1;
            const uint4 v = *reinterpret_cast<const uint4 *>(src + (size_t)row * kKsRow + c4);
            *reinterpret_cast<uint4 *>(&rows[ij * 4 + h][c4]) = v;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPerWave; ++k) {
            const int g = ct0 + wave * kPerWave + k;
            if (g >= B) break;                         // wave-uniform
            const int32_t *ua = u_a + (size_t)g * kN + i0;
            const int32_t *ua2 = u2_a ? u2_a + (size_t)g * kN + i0 : nullptr;
#pragma unroll
            for (int ii = 0; ii < kKsI; ++ii) {
                uint32_t ab = (uint32_t)__builtin_amdgcn_readfirstlane(ua[ii]);
                if (ua2) ab += (uint32_t)__builtin_amdgcn_readfirstlane(ua2[ii]);
                ab += kKsPrecOffset;
#pragma unroll
                for (int j = 0; j < kKsT; ++j) {
                    const uint32_t aij = (ab >> (32 - (j + 1) * kKsBasebit)) & (kKsBase - 1);
                    acc[k] -= rows[(ii * kKsT + j) * 4 + (int)aij][lane];
                }
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < kPerWave; ++k) {
        const int g = ct0 + wave * kPerWave + k;
        if (g >= B) break;
        if (col < kn) res_a[(size_t)g * kn + col] = (int32_t)acc[k];
        else if (col == kn) res_b[g] = (int32_t)acc[k];
    }
}

}  // namespace

int ks_version() {
    static const int v = [] {
        const char *e = getenv("TFHE_AMD_KS");
        return (e && atoi(e) == 1) ? 1 : 2;
    }();
    return v;
}

hipError_t launch_keyswitch(const DeviceKey &key, int B, const int32_t *u_a, const int32_t *u_b,
                            const int32_t *u2_a, const int32_t *u2_b, int32_t add_b,
                            int32_t *res_a, int32_t *res_b, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (ks_version() == 1) {
        hipLaunchKernelGGL(k_keyswitch_v1, dim3(B), dim3(kKsThreads), 0, s, key.ksk, u_a, u_b, u2_a, u2_b,
                           add_b, res_a, res_b);
    } else {
        const int blocks = ((B + kKsCt - 1) / kKsCt) * 8;
        hipLaunchKernelGGL(k_keyswitch_v2, dim3(blocks), dim3(kKsV2Threads), 0, s, key.ksk, B, u_a, u_b, u2_a,
                           u2_b, add_b, res_a, res_b);
    }
    return hipGetLastError();
}

}  // namespace tfhe_amd
