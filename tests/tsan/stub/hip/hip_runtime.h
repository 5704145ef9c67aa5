// Test-only stand-in for <hip/hip_runtime.h>: the host-side HIP API the library's host code calls
// (csrc/engine.cpp, tfhe_api.cpp, multi.cpp, circuit.cpp, engine.h's DeviceScope / StreamFence),
// implemented on the CPU so that code can be built with -fsanitize=thread and no GPU
// (tests/test_concurrency_tsan.py).  "Device memory" is host memory and the current device is per
// thread, as in HIP.  Streams are ASYNCHRONOUS: each stream is a worker thread that runs its queue
// of operations (copies, memsets, the CPU stand-in kernels of tests/tsan/stub_kernels.cpp, event
// records, waits on other streams' events) in order, so that a host thread reading a result before
// synchronizing on the stream or event that produced it — or two streams touching one buffer
// without an event between them — is a data race ThreadSanitizer reports.  Synchronous calls
// (hipMemcpy, hipMemset) act on the host thread at once, as on a non-blocking stream's host.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <set>
#include <thread>

typedef enum hipError_t {
    hipSuccess = 0,
    hipErrorInvalidValue = 1,
    hipErrorOutOfMemory = 2,
    hipErrorInvalidDevice = 101,
    hipErrorNoDevice = 100,
    hipErrorPeerAccessAlreadyEnabled = 704,
} hipError_t;
typedef enum hipMemcpyKind {
    hipMemcpyHostToHost = 0,
    hipMemcpyHostToDevice = 1,
    hipMemcpyDeviceToHost = 2,
    hipMemcpyDeviceToDevice = 3,
    hipMemcpyDefault = 4
} hipMemcpyKind;
struct uint2 { unsigned x, y; };
struct double2 { double x, y; };
inline double2 make_double2(double x, double y) { return double2{x, y}; }
inline uint2 make_uint2(unsigned x, unsigned y) { return uint2{x, y}; }
#define hipStreamNonBlocking 1
#define hipEventDisableTiming 2
#define hipHostMallocDefault 0
#define hipHostMallocPortable 1
#define hipHostMallocMapped 2

// one in-order queue of device work, run by its own thread
struct StubStream {
    int device = 0;
    std::mutex mu;
    std::condition_variable cv, idle_cv;
    std::deque<std::function<void()>> q;
    bool busy = false, stop = false;
    std::thread worker;
    explicit StubStream(int d) : device(d) {
        worker = std::thread([this] {
            std::unique_lock<std::mutex> lk(mu);
            for (;;) {
                cv.wait(lk, [&] { return stop || !q.empty(); });
                if (q.empty()) return;
                std::function<void()> f = std::move(q.front());
                q.pop_front();
                busy = true;
                lk.unlock();
                f();
                lk.lock();
                busy = false;
                if (q.empty()) idle_cv.notify_all();
            }
        });
    }
    void push(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> lk(mu);
            q.push_back(std::move(f));
        }
        cv.notify_one();
    }
    void drain() {
        std::unique_lock<std::mutex> lk(mu);
        idle_cv.wait(lk, [&] { return q.empty() && !busy; });
    }
    ~StubStream() {
        drain();
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        worker.join();
    }
};
struct StubEvent {
    std::mutex mu;
    std::condition_variable cv;
    uint64_t recorded = 0, completed = 0;
    void wait_for(uint64_t t) {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return completed >= t; });
    }
};
typedef StubStream *hipStream_t;
typedef StubEvent *hipEvent_t;

namespace hip_stub {
inline int &device_count() { static int n = 2; return n; }      // set by the test driver
inline int &current() { thread_local int d = 0; return d; }
inline std::atomic<long> &set_calls() { static std::atomic<long> n{0}; return n; }
inline std::mutex &reg_mu() { static std::mutex m; return m; }
inline std::set<StubStream *> &streams() { static std::set<StubStream *> s; return s; }
// the null stream: work enqueued on stream 0 (one per process, never destroyed)
inline StubStream *null_stream() {
    static StubStream *s = [] {
        StubStream *n = new StubStream(0);
        std::lock_guard<std::mutex> lk(reg_mu());
        streams().insert(n);
        return n;
    }();
    return s;
}
inline StubStream *of(hipStream_t s) { return s ? s : null_stream(); }
// enqueue device work (the stand-in kernels use this too)
inline void enqueue(hipStream_t s, std::function<void()> f) { of(s)->push(std::move(f)); }
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
// host memory is the device's in the stand-in: mapped at the same address
inline hipError_t hipHostGetDevicePointer(void **dp, void *p, unsigned) { *dp = p; return hipSuccess; }
inline hipError_t hipHostFree(void *p) { free(p); return hipSuccess; }
inline hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind) { if (n) memmove(d, s, n); return hipSuccess; }
inline hipError_t hipMemcpyAsync(void *d, const void *s, size_t n, hipMemcpyKind, hipStream_t st) {
    if (n) hip_stub::enqueue(st, [=] { memmove(d, s, n); });
    return hipSuccess;
}
inline hipError_t hipMemcpyPeerAsync(void *d, int, const void *s, int, size_t n, hipStream_t st) {
    return hipMemcpyAsync(d, s, n, hipMemcpyDeviceToDevice, st);
}
inline hipError_t hipMemcpy2DAsync(void *d, size_t dp, const void *s, size_t sp, size_t w, size_t h, hipMemcpyKind,
                                   hipStream_t st) {
    hip_stub::enqueue(st, [=] {
        for (size_t r = 0; r < h; ++r) memmove((char *)d + r * dp, (const char *)s + r * sp, w);
    });
    return hipSuccess;
}
inline hipError_t hipMemset(void *d, int v, size_t n) { memset(d, v, n); return hipSuccess; }
inline hipError_t hipMemsetAsync(void *d, int v, size_t n, hipStream_t st) {
    hip_stub::enqueue(st, [=] { memset(d, v, n); });
    return hipSuccess;
}
inline hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned) {
    *s = new StubStream(hip_stub::current());
    std::lock_guard<std::mutex> lk(hip_stub::reg_mu());
    hip_stub::streams().insert(*s);
    return hipSuccess;
}
inline hipError_t hipStreamDestroy(hipStream_t s) {
    {
        std::lock_guard<std::mutex> lk(hip_stub::reg_mu());
        hip_stub::streams().erase(s);
    }
    delete s;   // drains its queue first, as hipStreamDestroy lets pending work finish
    return hipSuccess;
}
inline hipError_t hipStreamSynchronize(hipStream_t s) { hip_stub::of(s)->drain(); return hipSuccess; }
inline hipError_t hipDeviceSynchronize() {
    std::lock_guard<std::mutex> lk(hip_stub::reg_mu());   // streams are not destroyed meanwhile
    for (StubStream *s : hip_stub::streams())
        if (s->device == hip_stub::current()) s->drain();
    return hipSuccess;
}
inline hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned) { *e = new StubEvent(); return hipSuccess; }
inline hipError_t hipEventCreate(hipEvent_t *e) { return hipEventCreateWithFlags(e, 0); }
inline hipError_t hipEventDestroy(hipEvent_t e) { delete e; return hipSuccess; }
inline hipError_t hipEventRecord(hipEvent_t e, hipStream_t st) {
    uint64_t t;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        t = ++e->recorded;
    }
    hip_stub::enqueue(st, [e, t] {
        {
            std::lock_guard<std::mutex> lk(e->mu);
            e->completed = std::max(e->completed, t);
        }
        e->cv.notify_all();
    });
    return hipSuccess;
}
inline hipError_t hipEventSynchronize(hipEvent_t e) {
    uint64_t t;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        t = e->recorded;
    }
    e->wait_for(t);
    return hipSuccess;
}
inline hipError_t hipEventElapsedTime(float *ms, hipEvent_t a, hipEvent_t b) {
    (void)hipEventSynchronize(a);
    (void)hipEventSynchronize(b);
    *ms = 0.5f;
    return hipSuccess;
}
inline hipError_t hipStreamWaitEvent(hipStream_t st, hipEvent_t e, unsigned) {
    uint64_t t;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        t = e->recorded;
    }
    hip_stub::enqueue(st, [e, t] { e->wait_for(t); });
    return hipSuccess;
}
enum hipDeviceAttribute_t { hipDeviceAttributeMultiprocessorCount = 63 };
inline hipError_t hipDeviceGetAttribute(int *v, hipDeviceAttribute_t, int) { *v = 256; return hipSuccess; }
inline hipError_t hipDeviceCanAccessPeer(int *can, int, int) { *can = 1; return hipSuccess; }
inline hipError_t hipDeviceEnablePeerAccess(int, unsigned) { return hipSuccess; }
