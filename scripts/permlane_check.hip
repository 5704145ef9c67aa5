// permlane_check.hip — the cross-lane swaps the radix-16 forward (fft_wave.h, v10) relies on,
// checked on the device against the semantics scripts/emu_v10.py assumes:
//   v_permlane32_swap(vdst = a, src = b): a's lanes 32..63 <-> b's lanes 0..31
//   v_permlane16_swap(vdst = a, src = b): a's odd rows (lanes 16..31, 48..63) <-> b's even rows
// Build: hipcc --offload-arch=gfx950 -O2 scripts/permlane_check.hip -o scripts/_bin/permlane_check
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned *out) {
    const unsigned L = threadIdx.x;
    const unsigned a = 1000 + L, b = 2000 + L;
    auto s32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    auto s16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    out[L] = s32[0];
    out[64 + L] = s32[1];
    out[128 + L] = s16[0];
    out[192 + L] = s16[1];
}

int main() {
    unsigned *d, h[256];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    for (unsigned L = 0; L < 64; ++L) {
        const unsigned a32 = L < 32 ? 1000 + L : 2000 + (L - 32);
        const unsigned b32 = L < 32 ? 1000 + (L + 32) : 2000 + L;
        const bool odd = (L >> 4) & 1;
        const unsigned a16 = odd ? 2000 + (L - 16) : 1000 + L;
        const unsigned b16 = odd ? 2000 + L : 1000 + (L + 16);
        bad += h[L] != a32;
        bad += h[64 + L] != b32;
        bad += h[128 + L] != a16;
        bad += h[192 + L] != b16;
    }
    printf("permlane_check: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
    if (bad)
        for (int L = 0; L < 64; L += 8)
            printf("L=%2d s32 %u %u  s16 %u %u\n", L, h[L], h[64 + L], h[128 + L], h[192 + L]);
    (void)hipFree(d);
    return bad ? 1 : 0;
}
