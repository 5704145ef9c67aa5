// mfma_i8_map.hip — checks the operand / result lane maps of v_mfma_i32_32x32x32_i8 with exact
// integer data (dev tool, GPU box).  Hypothesis: lane l (r = l & 31, h = l >> 5) holds
// A[r][16 h + j] and B[16 h + j][r] in byte j of its 16-byte fragments; C/D: col = l & 31,
// row = (reg & 3) + 8 (reg >> 2) + 4 h.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k(const signed char *A, const signed char *B, int *D) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    v4i a, b;
    signed char *pa = (signed char *)&a, *pb = (signed char *)&b;
    for (int j = 0; j < 16; ++j) {
        pa[j] = A[r * 32 + 16 * h + j];
        pb[j] = B[(16 * h + j) * 32 + r];
    }
    v16i c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    for (int reg = 0; reg < 16; ++reg) D[((reg & 3) + 8 * (reg >> 2) + 4 * h) * 32 + r] = c[reg];
}

int main() {
    signed char hA[32 * 32], hB[32 * 32];
    for (int i = 0; i < 32; ++i)
        for (int kk = 0; kk < 32; ++kk) {
            hA[i * 32 + kk] = (signed char)((i * 7 + kk * 3 + 1) % 255 - 127);
            hB[kk * 32 + i] = (signed char)((kk * 11 + i * 5 + 2) % 253 - 126);
        }
    signed char *dA, *dB;
    int *dD;
    (void)hipMalloc(&dA, 1024); (void)hipMalloc(&dB, 1024); (void)hipMalloc(&dD, 4096);
    (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    int hD[1024];
    (void)hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 32; ++i)
        for (int jj = 0; jj < 32; ++jj) {
            int s = 0;
            for (int kk = 0; kk < 32; ++kk) s += hA[i * 32 + kk] * hB[kk * 32 + jj];
            if (s != hD[i * 32 + jj]) ++bad;
        }
    printf("v_mfma_i32_32x32x32_i8 map check: %d of 1024 wrong\n", bad);
    return bad != 0;
}
