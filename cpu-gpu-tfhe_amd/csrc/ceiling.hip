// ceiling.hip — the fp64 FMA rate this GPU sustains under its power limit (measurement entry
// point for bench.py's roofline, not on the bootstrapping path).
//
// MI355X's 78.6 TFLOP/s fp64 vector peak assumes the 2.4 GHz peak clock; a chip that keeps
// every SIMD issuing fp64 FMAs runs into its 1 400 W socket limit first and lowers the clock
// (the blind rotation holds ~1 300 W).  This kernel measures the rate the chip
// actually sustains: every lane runs 16 independent v_fma_f64 chains on register operands with
// changing mantissas (random-like data: a zero-operand loop would draw less power), `waves`
// waves per SIMD, for about `seconds` of wall time after a short calibration launch.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

constexpr int kCeilThreads = 256;

__global__ __launch_bounds__(kCeilThreads) void k_fp64_ceiling(double *__restrict__ out, long iters,
                                                             unsigned long long *__restrict__ clk) {
    const unsigned t = blockIdx.x * kCeilThreads + threadIdx.x;
    double acc[16], b[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const unsigned h = (t * 2654435761u) ^ (j * 40503u + 0x9e3779b9u);
        acc[j] = 1.0 + (double)(h & 0xfffff) * 0x1p-21;
        b[j] = (double)((h >> 11) & 0xffff) * 0x1p-30 + 0x1p-12;
    }
    // |a| < 1: each chain converges to b / (1 - a) (~0.13..0.25) with all mantissa bits moving
    const double a = 0.984375 - (double)(t & 63) * 0x1p-20;
    unsigned long long c0 = 0, r0 = 0;
    if (t == 0) {
        c0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (long i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = __builtin_fma(acc[j], a, b[j]);
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += acc[j];
    out[t] = s;
    if (t == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - c0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

}  // namespace

// tflops: fp64 FLOP/s (FMA = 2) / 1e12 over the timed launch; mhz: shader clock of workgroup 0's
// CU over it (s_memtime / s_memrealtime at 100 MHz).  0 on success.
extern "C" int tfhe_amd_fp64_ceiling(int device, int waves_per_simd, double seconds, double *tflops, double *mhz) {
    if (!tflops || !mhz || waves_per_simd < 1 || waves_per_simd > 8 || !(seconds > 0.0) || seconds > 30.0) return -1;
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return -2;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) {
        (void)hipSetDevice(prev);
        return -2;
    }
    // 4 waves per workgroup, one per SIMD: waves_per_simd workgroups per CU
    const int blocks = cus * waves_per_simd;
    double *out = nullptr;
    unsigned long long *clk = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = -2;
    if (hipMalloc(&out, (size_t)blocks * kCeilThreads * sizeof(double)) != hipSuccess) goto done;
    if (hipMalloc(&clk, 2 * sizeof(unsigned long long)) != hipSuccess) goto done;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) goto done;
    {
        long iters = 20000;
        float ms = 0.f;
        for (int pass = 0; pass < 2; ++pass) {   // calibration, then the timed launch
            if (hipEventRecord(e0, nullptr) != hipSuccess) goto done;
            hipLaunchKernelGGL(k_fp64_ceiling, dim3(blocks), dim3(kCeilThreads), 0, nullptr, out, iters, clk);
            if (hipGetLastError() != hipSuccess || hipEventRecord(e1, nullptr) != hipSuccess) goto done;
            if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess || ms <= 0.f)
                goto done;
            if (pass == 0) {
                const double scale = seconds * 1000.0 / ms;
                iters = (long)((double)iters * (scale > 4000.0 ? 4000.0 : scale));
                if (iters < 1000) iters = 1000;
            }
        }
        const double flop = (double)blocks * kCeilThreads * (double)iters * 16.0 * 2.0;
        *tflops = flop / (ms * 1e-3) / 1e12;
        unsigned long long h[2] = {0, 0};
        if (hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) goto done;
        *mhz = h[1] ? (double)h[0] / ((double)h[1] / 100.0) : 0.0;
        rc = 0;
    }
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (out) (void)hipFree(out);
    if (clk) (void)hipFree(clk);
    (void)hipSetDevice(prev);   // the caller's current device is left as it was
    return rc;
}
