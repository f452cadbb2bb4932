// Times the HIP runtime's start-up steps as the saln CLI meets them
// (saln_context_create, first allocations, first copies), to see what the
// CLI leg's "context" stage is made of.
// Build: hipcc -O2 --offload-arch=gfx950 -x hip hip_init_time.cpp -o hip_init_time
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

namespace {
double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}
}  // namespace

int main() {
    double t = now_ms();
    auto mark = [&](const char *what, hipError_t e) {
        const double n = now_ms();
        std::printf("{\"step\": \"%s\", \"ms\": %.3f, \"ok\": %s}\n", what, n - t,
                    e == hipSuccess ? "true" : "false");
        t = n;
        if (e != hipSuccess) std::exit(1);
    };
    int n = 0;
    mark("hipGetDeviceCount", hipGetDeviceCount(&n));
    hipDeviceProp_t prop;
    mark("hipGetDeviceProperties", hipGetDeviceProperties(&prop, 0));
    mark("hipSetDevice", hipSetDevice(0));
    hipStream_t s1, s2;
    mark("hipStreamCreate x2", [&] {
        hipError_t e = hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
        return e != hipSuccess ? e : hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    }());
    void *d = nullptr;
    mark("hipMalloc 1 GB", hipMalloc(&d, 1ull << 30));
    void *h = nullptr;
    mark("hipHostMalloc 64 MB", hipHostMalloc(&h, 64ull << 20, 0));
    mark("H2D 64 MB pinned", [&] {
        hipError_t e = hipMemcpyAsync(d, h, 64ull << 20, hipMemcpyHostToDevice, s1);
        return e != hipSuccess ? e : hipStreamSynchronize(s1);
    }());
    mark("H2D 64 MB pinned again", [&] {
        hipError_t e = hipMemcpyAsync(d, h, 64ull << 20, hipMemcpyHostToDevice, s1);
        return e != hipSuccess ? e : hipStreamSynchronize(s1);
    }());
    void *p = std::malloc(16ull << 20);
    mark("H2D 16 MB pageable", hipMemcpy(d, p, 16ull << 20, hipMemcpyHostToDevice));
    mark("H2D 16 MB pageable again", hipMemcpy(d, p, 16ull << 20, hipMemcpyHostToDevice));
    mark("hipFree", hipFree(d));
    std::printf("{\"devices\": %d}\n", n);
    return 0;
}
