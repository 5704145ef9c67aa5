// Test-only stand-in for <hip/hip_runtime.h>: just the host-side HIP API that the library's
// concurrency code (csrc/tfhe_api.cpp, multi.cpp, circuit.cpp, engine.h's DeviceScope /
// StreamFence) calls, implemented on the CPU so that code can be built with
// -fsanitize=thread and no GPU (tests/test_concurrency_tsan.py).  Streams and events are
// plain objects; "device memory" is host memory; the current device is per thread, as in HIP.
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>

typedef enum hipError_t {
    hipSuccess = 0,
    hipErrorInvalidValue = 1,
    hipErrorOutOfMemory = 2,
    hipErrorInvalidDevice = 101,
    hipErrorNoDevice = 100,
} hipError_t;
typedef enum hipMemcpyKind {
    hipMemcpyHostToHost = 0,
    hipMemcpyHostToDevice = 1,
    hipMemcpyDeviceToHost = 2,
    hipMemcpyDeviceToDevice = 3,
    hipMemcpyDefault = 4
} hipMemcpyKind;
struct StubStream { int device; };
struct StubEvent { std::atomic<int> recorded{0}; };
typedef StubStream *hipStream_t;
typedef StubEvent *hipEvent_t;
struct uint2 { unsigned x, y; };
struct double2 { double x, y; };
inline double2 make_double2(double x, double y) { return double2{x, y}; }
#define hipStreamNonBlocking 1
#define hipEventDisableTiming 2
#define hipHostMallocDefault 0

namespace hip_stub {
inline int &device_count() { static int n = 2; return n; }      // set by the test driver
inline int &current() { thread_local int d = 0; return d; }
inline std::atomic<long> &set_calls() { static std::atomic<long> n{0}; return n; }
}  // namespace hip_stub

inline hipError_t hipGetDeviceCount(int *n) { *n = hip_stub::device_count(); return hipSuccess; }
inline hipError_t hipGetDevice(int *d) { *d = hip_stub::current(); return hipSuccess; }
inline hipError_t hipSetDevice(int d) {
    if (d < 0 || d >= hip_stub::device_count()) return hipErrorInvalidDevice;
    hip_stub::set_calls()++;
    hip_stub::current() = d;
    return hipSuccess;
}
inline const char *hipGetErrorString(hipError_t) { return "stub"; }
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipMalloc(void **p, size_t n) { *p = calloc(1, n ? n : 1); return *p ? hipSuccess : hipErrorOutOfMemory; }
template <class T> inline hipError_t hipMalloc(T **p, size_t n) { return hipMalloc((void **)p, n); }
inline hipError_t hipFree(void *p) { free(p); return hipSuccess; }
inline hipError_t hipHostMalloc(void **p, size_t n, unsigned) { return hipMalloc(p, n); }
template <class T> inline hipError_t hipHostMalloc(T **p, size_t n, unsigned f) { return hipHostMalloc((void **)p, n, f); }
inline hipError_t hipHostFree(void *p) { free(p); return hipSuccess; }
inline hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind) { if (n) memmove(d, s, n); return hipSuccess; }
inline hipError_t hipMemcpyAsync(void *d, const void *s, size_t n, hipMemcpyKind k, hipStream_t) { return hipMemcpy(d, s, n, k); }
inline hipError_t hipMemcpy2DAsync(void *d, size_t dp, const void *s, size_t sp, size_t w, size_t h, hipMemcpyKind,
                                   hipStream_t) {
    for (size_t r = 0; r < h; ++r) memmove((char *)d + r * dp, (const char *)s + r * sp, w);
    return hipSuccess;
}
inline hipError_t hipMemset(void *d, int v, size_t n) { memset(d, v, n); return hipSuccess; }
inline hipError_t hipMemsetAsync(void *d, int v, size_t n, hipStream_t) { memset(d, v, n); return hipSuccess; }
inline hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned) { *s = new StubStream{hip_stub::current()}; return hipSuccess; }
inline hipError_t hipStreamDestroy(hipStream_t s) { delete s; return hipSuccess; }
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
inline hipError_t hipDeviceSynchronize() { return hipSuccess; }
inline hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned) { *e = new StubEvent(); return hipSuccess; }
inline hipError_t hipEventCreate(hipEvent_t *e) { return hipEventCreateWithFlags(e, 0); }
inline hipError_t hipEventDestroy(hipEvent_t e) { delete e; return hipSuccess; }
inline hipError_t hipEventRecord(hipEvent_t e, hipStream_t) { e->recorded++; return hipSuccess; }
inline hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
inline hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }
