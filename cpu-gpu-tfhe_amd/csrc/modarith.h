// modarith.h — device-side modular arithmetic for the exact external product (q < 2^30).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "params.h"
#include "ntt_tables.h"

namespace tfhe_amd {

constexpr uint32_t kQ0 = 134215681u;
constexpr uint32_t kQ1 = 134203393u;
static_assert(kQ0 == kQ[0] && kQ1 == kQ[1], "prime mismatch");

__device__ __forceinline__ uint32_t q_of(int s) { return s ? kQ1 : kQ0; }

// a * w mod q for any a < 2^32 and w < q (Shoup, wp = floor(w 2^32 / q)); result in [0, q)
__device__ __forceinline__ uint32_t mul_shoup(uint32_t a, uint32_t w, uint32_t wp, uint32_t q) {
    const uint32_t qh = __umulhi(a, wp);
    const uint32_t r = a * w - qh * q;
    return r >= q ? r - q : r;
}
// lazy variant: result in [0, 2q)
__device__ __forceinline__ uint32_t mul_shoup_lazy(uint32_t a, uint32_t w, uint32_t wp, uint32_t q) {
    const uint32_t qh = __umulhi(a, wp);
    return a * w - qh * q;
}
__device__ __forceinline__ uint32_t add_mod(uint32_t a, uint32_t b, uint32_t q) {
    const uint32_t s = a + b;
    return s >= q ? s - q : s;
}
__device__ __forceinline__ uint32_t sub_mod(uint32_t a, uint32_t b, uint32_t q) {
    const uint32_t s = a + q - b;
    return s >= q ? s - q : s;
}
// Montgomery REDC: x < q 2^32  ->  x 2^-32 mod q, in [0, q)
__device__ __forceinline__ uint32_t redc(uint64_t x, uint32_t q, uint32_t qinv_neg) {
    const uint32_t m = (uint32_t)x * qinv_neg;
    const uint32_t r = (uint32_t)((x + (uint64_t)m * q) >> 32);
    return r >= q ? r - q : r;
}
// signed digit d in (-q, q) -> [0, q)
__device__ __forceinline__ uint32_t digit_mod(int32_t d, uint32_t q) {
    return d < 0 ? (uint32_t)(d + (int32_t)q) : (uint32_t)d;
}
// centred CRT lift of (x0 mod q0, x1 mod q1), reduced mod 2^32 (the Torus32 result)
__device__ __forceinline__ uint32_t crt_torus(uint32_t x0, uint32_t x1, uint32_t h, uint32_t hp) {
    const uint32_t x0r = x0 >= kQ1 ? x0 - kQ1 : x0;
    const uint32_t d = sub_mod(x1, x0r, kQ1);
    const uint32_t t = mul_shoup(d, h, hp, kQ1);
    const uint64_t M = (uint64_t)kQ0 * kQ1;
    uint64_t X = (uint64_t)x0 + (uint64_t)kQ0 * t;
    if (X > (M >> 1)) X -= M;
    return (uint32_t)X;
}
// modSwitchFromTorus32(x, 2N) (numeric-functions.cu:60-66).  The reference computes
// (x << 32) + 2^52 in uint64_t, which wraps for x in [2^32 - 2^20, 2^32): those phases give
// 0, never 2N.  Equivalently: floor((x + 2^20) / 2^21) mod 2N.
__device__ __forceinline__ int modswitch_2N(uint32_t x) {
    return (int)((((uint64_t)x + (1u << 20)) >> 21) & (k2N - 1));
}

}  // namespace tfhe_amd
