// ubench_fp64.hip — fp64 VALU issue-rate probes (dev tool, GPU box): rate of v_fma_f64 chains by
// operand form and waves per SIMD.  hipcc --offload-arch=gfx950 -O3 -o ubench_fp64 ubench_fp64.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int MODE>
__global__ __launch_bounds__(256) void k(double *out, long iters, double sa, double sb) {
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    double acc[16], b[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const unsigned h = (t * 2654435761u) ^ (j * 40503u + 0x9e3779b9u);
        acc[j] = 1.0 + (double)(h & 0xfffff) * 0x1p-21;
        b[j] = (double)((h >> 11) & 0xffff) * 0x1p-30 + 0x1p-12;
    }
    const double a = 0.984375 - (double)(t & 63) * 0x1p-20;
    for (long i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (MODE == 0) acc[j] = __builtin_fma(acc[j], a, b[j]);          // 3 VGPR pairs
            else if (MODE == 1) acc[j] = __builtin_fma(acc[j], sa, sb);      // 1 VGPR pair + SGPRs
            else if (MODE == 2) acc[j] = __builtin_fma(acc[j], a, sb);       // 2 VGPR pairs + SGPR
            else if (MODE == 3) acc[j] = acc[j] * sa + b[j] * 0.0 + sb;     // (compiler decides)
            else acc[j] = acc[j] + b[j];                                     // v_add_f64, 2 pairs
        }
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += acc[j];
    out[t] = s;
}

template <int MODE>
static void run(int cus, int w, double *out) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const long iters = 200000;
    const int blocks = cus * w;
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.984375, 0x1p-12);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
    }
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double ops = (double)blocks * 256 * iters * 16;   // fp64 instructions x lanes
    printf("mode %d waves/SIMD %d: %.1f G lane-ops/s = %.1f TFLOP/s (FMA=2)\n", MODE, w, ops / ms / 1e6, 2 * ops / ms / 1e9);
}

int main() {
    int cus; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    double *out; hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(double));
    for (int w : {1, 2, 4}) { run<0>(cus, w, out); run<1>(cus, w, out); run<2>(cus, w, out); run<4>(cus, w, out); }
    return 0;
}
