// ubench_int.hip — issue cost of the integer VALU ops the exact NTT is built from (gfx950).
// Each thread runs 8 independent chains of ONE instruction forced by inline asm (so the
// compiler cannot strength-reduce the chain); prints SIMD-cycles per wave64 instruction
// assuming 1024 SIMDs at 2.4 GHz (relative numbers are what matter).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CH 8
#define ITERS 2048

#define OP1(ins) asm volatile(ins " %0, %0, %1" : "+v"(x[c]) : "v"(y[c]))

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t *out, uint32_t seed) {
    uint32_t x[CH], y[CH];
    uint64_t z[CH];
    for (int c = 0; c < CH; c++) {
        x[c] = seed * (threadIdx.x + c + 1);
        y[c] = x[c] ^ 0x9e3779b9u;
        z[c] = ((uint64_t)x[c] << 32) | y[c];
    }
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            if (OP == 0) OP1("v_mul_lo_u32");
            if (OP == 1) OP1("v_mul_hi_u32");
            if (OP == 2) OP1("v_mul_u32_u24");
            if (OP == 3) OP1("v_mul_hi_u32_u24");
            if (OP == 4) OP1("v_add_u32");
            if (OP == 5) OP1("v_min_u32");
            if (OP == 6) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(z[c]) : "v"(x[c]), "v"(y[c]) : "vcc");
            if (OP == 7) asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(x[c]) : "v"(y[c]));
            if (OP == 8) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x[c]) : "v"(y[c]));
            if (OP == 9) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(x[c]) : "v"(y[c]));
            if (OP == 10) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y[c]));
            if (OP == 11) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(z[c]));
            if (OP == 12) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x[c]) : "v"(y[c]));
        }
    }
    uint32_t r = 0;
    for (int c = 0; c < CH; c++) r ^= x[c] ^ (uint32_t)z[c] ^ (uint32_t)(z[c] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
void run(const char *name, uint32_t *d, int blocks) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, d, 12345u);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, d, 12345u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    double ops = (double)blocks * 256 * CH * ITERS;
    double wave_instr_per_simd = ops / 64.0 / 1024.0;
    double cycles = ms * 1e-3 * 2.4e9;
    printf("%-20s %9.1f Gop/s  %6.2f SIMD-cycles/wave-instr\n", name, ops / (ms * 1e-3) / 1e9,
           cycles / wave_instr_per_simd);
}

int main() {
    uint32_t *d;
    int blocks = 256 * 8;
    (void)hipMalloc(&d, sizeof(uint32_t) * blocks * 256);
    run<0>("v_mul_lo_u32", d, blocks);
    run<1>("v_mul_hi_u32", d, blocks);
    run<2>("v_mul_u32_u24", d, blocks);
    run<3>("v_mul_hi_u32_u24", d, blocks);
    run<4>("v_add_u32", d, blocks);
    run<10>("v_sub_u32", d, blocks);
    run<5>("v_min_u32", d, blocks);
    run<6>("v_mad_u64_u32", d, blocks);
    run<7>("v_alignbit_b32", d, blocks);
    run<8>("v_add3_u32", d, blocks);
    run<9>("v_mad_u32_u24", d, blocks);
    run<12>("v_lshl_add_u32", d, blocks);
    run<11>("v_fma_f64", d, blocks);
    (void)hipFree(d);
    return 0;
}
