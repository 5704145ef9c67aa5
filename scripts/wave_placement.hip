// Where the dispatcher puts the waves of a v6-shaped launch (dev tool): 128-thread workgroups
// holding ~37 KB of LDS (the blind rotation's footprint, plus an optional pad), each wave records
// its HW_ID / XCC_ID and then spins on fp64 FMAs long enough that the whole grid is resident.
// Prints, per grid size, how many waves share a SIMD and how many workgroups share a CU.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/wave_placement scripts/wave_placement.hip
//   scripts/wave_placement [pad_bytes]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

template <int T>
__global__ __launch_bounds__(T) void k_place(unsigned *out, double *sink, int iters) {
    __shared__ double lds[4600 * (T / 128)];   // 36.8 KB per ciphertext, like V6Shared
    extern __shared__ double pad[];
    const int w = threadIdx.x >> 6, L = threadIdx.x & 63;
    constexpr int W = T / 64;
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (L == 0) {
        out[4 * (blockIdx.x * W + w) + 0] = hw;
        out[4 * (blockIdx.x * W + w) + 1] = xcc;
    }
    lds[threadIdx.x] = threadIdx.x;
    pad[0] = 0.0;
    __syncthreads();
    double a = lds[(threadIdx.x + 1) & 127], b = 1.0000001, c = 0.5;
    for (int i = 0; i < iters; ++i) {
        a = fma(a, b, c);
        c = fma(c, b, a);
    }
    if (a == 12345.678) sink[threadIdx.x] = a + c;
}

template <int T>
static void run(int pad) {
    constexpr int W = T / 64;
    CHECK(hipFuncSetAttribute((const void *)k_place<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - 36800 * (T / 128)));
    const int sizes[] = {64, 256, 512, 768, 1024};
    unsigned *d_out;
    double *d_sink;
    CHECK(hipMalloc(&d_out, 1024 * 4 * 4 * sizeof(unsigned)));
    CHECK(hipMalloc(&d_sink, 256 * sizeof(double)));
    for (int B0 : sizes) {
        const int B = B0 / (T / 128);   // workgroups for B0 ciphertexts
        CHECK(hipMemset(d_out, 0, 1024 * 4 * 4 * sizeof(unsigned)));
        hipLaunchKernelGGL(k_place<T>, dim3(B), dim3(T), pad + 8, 0, d_out, d_sink, 200000);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        std::vector<unsigned> h(B * W * 4);
        CHECK(hipMemcpy(h.data(), d_out, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
        std::map<unsigned, int> per_simd, per_cu_waves;
        std::map<unsigned, std::map<int, int>> cu_wgs;
        int same_simd_pairs = 0;
        for (int g = 0; g < B; ++g) {
            unsigned simd_key[W];
            for (int w = 0; w < W; ++w) {
                const unsigned hw = h[4 * (W * g + w)], xcc = h[4 * (W * g + w) + 1] & 0xF;
                const unsigned cu = (xcc << 16) | (((hw >> 13) & 0x7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF);
                const unsigned simd = (cu << 2) | ((hw >> 4) & 3);
                simd_key[w] = simd;
                per_simd[simd]++;
                per_cu_waves[cu]++;
                cu_wgs[cu][g] = 1;
            }
            same_simd_pairs += simd_key[0] == simd_key[1];
        }
        std::map<int, int> hs, hc;
        for (auto &kv : per_simd) hs[kv.second]++;
        for (auto &kv : cu_wgs) hc[(int)kv.second.size()]++;
        printf("T=%d cts=%d wgs=%d pad=%d: CUs %zu, SIMDs %zu; workgroups with both waves on one SIMD %d\n", T, B0, B, pad,
               per_cu_waves.size(), per_simd.size(), same_simd_pairs);
        printf("  waves per occupied SIMD:");
        for (auto &kv : hs) printf(" %d:%d", kv.first, kv.second);
        printf("\n  workgroups per occupied CU:");
        for (auto &kv : hc) printf(" %d:%d", kv.first, kv.second);
        printf("\n");
    }
    CHECK(hipFree(d_out));
    CHECK(hipFree(d_sink));
}

int main(int argc, char **argv) {
    const int pad = argc > 1 ? atoi(argv[1]) : 0;
    run<128>(pad);
    run<256>(pad);
    return 0;
}
