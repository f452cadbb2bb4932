// Does hipExtAnyOrderLaunch let a kernel start before the previous kernel of
// the same stream has finished on gfx950?  Two spin kernels of ~1 ms each on
// one stream (a few waves, so both fit at once); the wall time of the pair is
// ~2 ms when the second waits for the first and ~1 ms when they overlap.
// Also times the gap an event record / cross-stream wait / timing events
// (recorded around a kernel, or given to hipExtLaunchKernel) leave between two
// short kernels.
// Build: hipcc -O2 --offload-arch=gfx950 anyorder.hip -o anyorder
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

__global__ void spin(uint64_t cycles, uint32_t *out) {
    const uint64_t t0 = wall_clock64();
    uint32_t x = threadIdx.x;
    while (wall_clock64() - t0 < cycles) x = x * 1664525u + 1013904223u;
    if (x == 0xFFFFFFFFu) out[0] = x;  // keeps the loop
}

#define CK(e)                                                                   \
    do {                                                                        \
        hipError_t r_ = (e);                                                    \
        if (r_ != hipSuccess) {                                                 \
            std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(r_)); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
    hipStream_t s, t;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
    uint32_t *out;
    CK(hipMalloc(&out, 64));
    // ~1 ms of the 100 MHz constant clock (wall_clock64)
    const uint64_t cyc = 100000;
    void *args[] = {(void *)&cyc, (void *)&out};
    for (int rep = 0; rep < 3; ++rep) {
        for (int flags = 0; flags < 2; ++flags) {
            CK(hipDeviceSynchronize());
            auto t0 = std::chrono::steady_clock::now();
            for (int k = 0; k < 4; ++k)
                CK(hipExtLaunchKernel((const void *)spin, dim3(8), dim3(64), args, 0, s, nullptr,
                                      nullptr, flags ? hipExtAnyOrderLaunch : 0));
            CK(hipStreamSynchronize(s));
            std::printf("{\"test\": \"4 spin kernels, one stream\", \"any_order\": %d, \"ms\": %.3f}\n",
                        flags, ms_since(t0));
        }
        // gaps between 200 short kernels: back to back / a marker between / a
        // cross-stream wait between
        hipEvent_t e;
        CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        const uint64_t shortc = 1000;  // ~10 us
        void *sargs[] = {(void *)&shortc, (void *)&out};
        hipEvent_t te[2];
        CK(hipEventCreate(&te[0]));
        CK(hipEventCreate(&te[1]));
        for (int mode = 0; mode < 5; ++mode) {
            CK(hipDeviceSynchronize());
            auto t0 = std::chrono::steady_clock::now();
            for (int k = 0; k < 200; ++k) {
                if (mode == 4) CK(hipEventRecord(te[0], s));
                CK(hipExtLaunchKernel((const void *)spin, dim3(8), dim3(64), sargs, 0, s,
                                      mode == 3 ? te[0] : nullptr, mode == 3 ? te[1] : nullptr, 0));
                if (mode == 4) CK(hipEventRecord(te[1], s));
                if (mode == 1) CK(hipEventRecord(e, s));
                if (mode == 2) {
                    CK(hipEventRecord(e, t));
                    CK(hipStreamWaitEvent(s, e, 0));
                }
            }
            CK(hipStreamSynchronize(s));
            const char *name[] = {"back to back", "event record between", "cross-stream wait between",
                                  "start/stop events of hipExtLaunchKernel",
                                  "timing events recorded around each"};
            std::printf("{\"test\": \"200 x 10 us kernels, %s\", \"us_per_kernel\": %.2f}\n", name[mode],
                        ms_since(t0) * 1000.0 / 200);
        }
        float ms = 0;
        CK(hipEventElapsedTime(&ms, te[0], te[1]));
        std::printf("{\"test\": \"last timed kernel\", \"us\": %.2f}\n", ms * 1000.0f);
        CK(hipEventDestroy(e));
        CK(hipEventDestroy(te[0]));
        CK(hipEventDestroy(te[1]));
    }
    return 0;
}
