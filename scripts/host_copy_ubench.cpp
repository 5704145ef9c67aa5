// Host-side copy alternatives for the host-pointer batch path: time to move a
// batch's inputs (nin x B x 501 int32 from ordinary pageable caller memory) into device memory
// and B x 501 results back, by
//   stage  : memcpy into pinned (1 thread) + one hipMemcpyAsync      (the round-3 path)
//   stageT : the same memcpy split over T threads
//   page   : hipMemcpyAsync straight from / to the pageable arrays
//   reg    : hipHostRegister the caller's arrays, hipMemcpyAsync, hipHostUnregister
// build: hipcc -O2 -fopenmp scripts/host_copy_ubench.cpp -o scripts/host_copy_ubench
#include <hip/hip_runtime.h>
#include <omp.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char **argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 1024;
    const size_t in_bytes = (size_t)2 * B * 501 * 4, out_bytes = (size_t)B * 501 * 4;
    std::vector<char> src(in_bytes), dst(out_bytes);
    memset(src.data(), 1, in_bytes);
    memset(dst.data(), 2, out_bytes);
    char *pin, *d;
    CK(hipHostMalloc((void **)&pin, in_bytes + out_bytes, hipHostMallocDefault));
    CK(hipMalloc((void **)&d, in_bytes + out_bytes));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto run = [&](const char *name, auto fn) {
        fn();
        double best = 1e9, tot = 0;
        for (int i = 0; i < 20; ++i) {
            const double t0 = now();
            fn();
            const double t = now() - t0;
            best = t < best ? t : best;
            tot += t;
        }
        printf("{\"B\": %d, \"method\": \"%s\", \"in_MB\": %.2f, \"out_MB\": %.2f, \"best_ms\": %.3f, \"mean_ms\": %.3f}\n", B,
               name, in_bytes / 1e6, out_bytes / 1e6, best * 1e3, tot / 20 * 1e3);
    };
    for (int T : {1, 2, 4, 8}) {
        char nm[32];
        snprintf(nm, sizeof nm, "stage%d", T);
        run(nm, [&] {
#pragma omp parallel for num_threads(T)
            for (int t = 0; t < T; ++t) {
                const size_t lo = in_bytes * t / T, hi = in_bytes * (t + 1) / T;
                memcpy(pin + lo, src.data() + lo, hi - lo);
            }
            CK(hipMemcpyAsync(d, pin, in_bytes, hipMemcpyHostToDevice, s));
            CK(hipMemcpyAsync(pin + in_bytes, d + in_bytes, out_bytes, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
#pragma omp parallel for num_threads(T)
            for (int t = 0; t < T; ++t) {
                const size_t lo = out_bytes * t / T, hi = out_bytes * (t + 1) / T;
                memcpy(dst.data() + lo, pin + in_bytes + lo, hi - lo);
            }
        });
    }
    run("page", [&] {
        CK(hipMemcpyAsync(d, src.data(), in_bytes, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(dst.data(), d + in_bytes, out_bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    });
    run("reg", [&] {
        CK(hipHostRegister(src.data(), in_bytes, hipHostRegisterDefault));
        CK(hipHostRegister(dst.data(), out_bytes, hipHostRegisterDefault));
        CK(hipMemcpyAsync(d, src.data(), in_bytes, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(dst.data(), d + in_bytes, out_bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        CK(hipHostUnregister(src.data()));
        CK(hipHostUnregister(dst.data()));
    });
    run("dma_only", [&] {
        CK(hipMemcpyAsync(d, pin, in_bytes, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(pin + in_bytes, d + in_bytes, out_bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    });
    return 0;
}
