// bar_probe.hip — can the host write device memory directly (large BAR), and
// what does a host -> GPU doorbell cost that way, against the worker's model
// (the GPU polls a word in pinned host memory over PCIe)?
//
//   bar_probe MODE [iters]
//   MODE 0: doorbell in pinned host memory, GPU polls it over PCIe (the
//           persistent worker's protocol today)
//   MODE 1: doorbell in fine-grained device memory (hipDeviceMallocFinegrained)
//           written by the host through the BAR, GPU polls its own HBM
//   MODE 2: as 1 with hipDeviceMallocUncached
// Each iteration: the host stores i into the doorbell, the GPU (one wave)
// sees it and stores i into a completion word in pinned host memory, the
// host spins on that.  Prints one JSON line: mode, round trip ns.
// A mode whose memory the host cannot write dies with SIGSEGV (run each mode
// as its own process).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

__global__ void pong(volatile uint32_t *bell, uint32_t *done, uint32_t iters)
{
    if (threadIdx.x != 0)
        return;
    for (uint32_t i = 1; i <= iters; ++i) {
        uint64_t spins = 0;
        while (__hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != i) {
            if (++spins > (1ull << 26))
                return;   // bounded: the host stopped
            __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(done, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const uint32_t iters = argc > 2 ? (uint32_t)atoi(argv[2]) : 20000u;
    uint32_t *done = nullptr, *bell = nullptr, *dbell = nullptr;
    if (hipHostMalloc((void **)&done, 64, hipHostMallocCoherent) != hipSuccess)
        return 2;
    *done = 0;
    hipError_t e = hipSuccess;
    if (mode == 0) {
        e = hipHostMalloc((void **)&bell, 64, hipHostMallocCoherent);
        if (e == hipSuccess)
            e = hipHostGetDevicePointer((void **)&dbell, bell, 0);
    } else {
        e = hipExtMallocWithFlags((void **)&bell, 64,
                                  mode == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached);
        dbell = bell;
    }
    if (e != hipSuccess) {
        printf("{\"tool\": \"bar_probe\", \"mode\": %d, \"alloc\": \"%s\"}\n", mode,
               hipGetErrorString(e));
        return 0;
    }
    if (mode != 0 && hipMemset(bell, 0, 64) != hipSuccess)
        return 3;
    if (mode == 0)
        *bell = 0;
    hipDeviceSynchronize();
    uint32_t *ddone = nullptr;
    if (hipHostGetDevicePointer((void **)&ddone, done, 0) != hipSuccess)
        return 4;
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, s, (volatile uint32_t *)dbell, ddone, iters);
    // first host store into the doorbell: SIGSEGV here if the host cannot
    // reach that memory
    volatile uint32_t *hb = bell;
    double t0 = 0;
    for (uint32_t i = 1; i <= iters; ++i) {
        if (i == 101)
            t0 = now();   // 100 warm-up round trips
        __atomic_store_n((uint32_t *)hb, i, __ATOMIC_RELEASE);
        uint64_t spins = 0;
        while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != i) {
            if (++spins > (1ull << 32)) {
                printf("{\"tool\": \"bar_probe\", \"mode\": %d, \"stuck_at\": %u}\n", mode, i);
                return 5;
            }
            __builtin_ia32_pause();
        }
    }
    const double dt = now() - t0;
    hipStreamSynchronize(s);
    printf("{\"tool\": \"bar_probe\", \"mode\": %d, \"round_trip_ns\": %.0f}\n", mode,
           dt / (iters - 100) * 1e9);
    return 0;
}
