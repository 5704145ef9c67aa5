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

}  // namespace

hipError_t launch_keyswitch(const DeviceKey &key, int B, const int32_t *u_a, const int32_t *u_b,
                            const int32_t *u2_a, const int32_t *u2_b, int32_t add_b,
                            int32_t *res_a, int32_t *res_b, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_keyswitch_v1, dim3(B), dim3(kKsThreads), 0, s, key.ksk, u_a, u_b, u2_a, u2_b,
                       add_b, res_a, res_b);
    return hipGetLastError();
}

}  // namespace tfhe_amd
