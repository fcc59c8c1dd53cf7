// hbm_sector.hip — measurement helper (not part of the product): does reading
// only part of each 64-byte packet window save HBM time on this box?  The
// reference's decision for an unhashed packet (UDP, IPv6, ARP, ...) needs bytes
// 12..23 of the frame only (ff_dpdk_if.c:1959-1981), all inside the window's
// first 32 bytes; a hashed TCP packet needs bytes 26..37 as well.
//
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_sector.hip -o tools/hbm_sector && tools/hbm_sector [MiB]
//
// Four rotating buffers (the MALL holds none of them between launches).  Every
// variant reads `part` bytes of every `rec`-byte record, lane-contiguous 16-byte
// loads; one JSON line per variant: µs per launch, records/µs, GB/s of bytes read.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

// PER = 16-byte pieces read per record, REC = 16-byte pieces per record
template <int PER, int REC, int U>
__global__ __launch_bounds__(512) void rd_part(const u32x4 *a, size_t nrec, uint32_t *sink)
{
    const size_t nload = nrec * PER;
    const size_t T = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t x = 0;
    for (; i + (U - 1) * T < nload; i += U * T) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = i + u * T;
            v[u] = __builtin_nontemporal_load(a + (j / PER) * REC + (j % PER));
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < nload; i += T) {
        const u32x4 v = __builtin_nontemporal_load(a + (i / PER) * REC + (i % PER));
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x9E3779B9u)
        sink[0] = x;
}

// The parse kernel's shape: persistent waves, chunk deal of 4 tiles, per
// 64-packet tile the lane loads piece (l % P) of packet tile*64 + k*(64/P) + l/P;
// P = 4 (whole window) or 2 (first 32 bytes).  Writes 6 B/pkt (q, hash) per tile
// like the probe; loads one tile ahead.
template <int P>
__global__ __launch_bounds__(512) void pkt_part(const u32x4 *win, const uint16_t *len, int16_t *q,
                                                uint32_t *hash, uint32_t n)
{
    constexpr int C = 4;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t W = gridDim.x * 8u;
    const uint32_t gw = blockIdx.x * 8u + (threadIdx.x >> 6);
    const uint32_t ntiles = (n + 63u) / 64u;
    const uint32_t nchunk = (ntiles + C - 1) / C;
    u32x4 nx[P];
    uint16_t nl = 0;
    auto issue = [&](uint32_t t0) {
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const uint32_t p = t0 + (64u / P) * k + lane / P;
            nx[k] = __builtin_nontemporal_load(win + (size_t)min(p, n - 1u) * 4u + (lane % P));
        }
        nl = len[min(t0 + lane, n - 1u)];
    };
    for (uint32_t c = gw; c < nchunk; c += W) {
        const uint32_t tb = c * C, te = min(tb + C, ntiles);
        issue(tb * 64u);
        for (uint32_t t = tb; t < te; ++t) {
            const uint32_t t0 = t * 64u;
            u32x4 cur[P];
#pragma unroll
            for (int k = 0; k < P; ++k)
                cur[k] = nx[k];
            const uint16_t cl = nl;
            if (t + 1 < te)
                issue(t0 + 64u);
            uint32_t x = cl;
#pragma unroll
            for (int k = 0; k < P; ++k)
                x ^= cur[k].x ^ cur[k].y ^ cur[k].z ^ cur[k].w;
            const uint32_t p = t0 + lane;
            if (p < n) {
                q[p] = (int16_t)(x & 0x7fff);
                hash[p] = x;
            }
        }
    }
}

template <typename F>
static float time_us(F f, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r)
        f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / reps;
}

int main(int argc, char **argv)
{
    const size_t mib = argc > 1 ? strtoul(argv[1], 0, 10) : 1024;
    const size_t bytes = mib << 20;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    u32x4 *a;
    uint32_t *sink, *h;
    uint16_t *len;
    int16_t *q;
    const uint32_t npk = (uint32_t)(bytes / 64);
    CK(hipMalloc(&a, bytes * 4));
    CK(hipMalloc(&sink, 4));
    CK(hipMalloc(&len, npk * 2ull * 4));
    CK(hipMalloc(&q, npk * 2ull * 4));
    CK(hipMalloc(&h, npk * 4ull * 4));
    CK(hipMemset(a, 1, bytes * 4));
    CK(hipMemset(len, 0, npk * 2ull * 4));
    const int reps = 20;
    int r = 0;
    auto buf = [&]() { return a + (size_t)(r++ % 4) * (bytes / 16); };
    auto rep = [&](const char *name, size_t nrec, double rd, float us) {
        printf("{\"variant\": \"%s\", \"us\": %.2f, \"Mrec_per_ms\": %.1f, \"GBps_read\": %.1f}\n", name, us,
               nrec / us / 1e3, rd / us / 1e3);
        fflush(stdout);
    };
    for (int pass = 0; pass < 2; ++pass) {
#define R(PER, REC, label)                                                                        \
        {                                                                                         \
            const size_t nrec = bytes / (16 * REC);                                               \
            rep(label, nrec, 16.0 * PER * nrec,                                                   \
                time_us([&] { rd_part<PER, REC, 4><<<cus * 2, 512>>>(buf(), nrec, sink); }, reps)); \
        }
        R(4, 4, "rec64 read 64 (all)")
        R(2, 4, "rec64 read first 32")
        R(1, 4, "rec64 read first 16")
        R(4, 8, "rec128 read first 64")
        R(2, 8, "rec128 read first 32")
#undef R
        const unsigned blocks = (unsigned)cus;
        rep("pkt shape P=4 (64 B window + len, 6 B out)", npk, 66.0 * npk,
            time_us([&] { const int k = r++ % 4; pkt_part<4><<<blocks, 512>>>(a + (size_t)k * (bytes / 16), len + (size_t)k * npk, q + (size_t)k * npk, h + (size_t)k * npk, npk); }, reps));
        rep("pkt shape P=2 (first 32 B + len, 6 B out)", npk, 34.0 * npk,
            time_us([&] { const int k = r++ % 4; pkt_part<2><<<blocks, 512>>>(a + (size_t)k * (bytes / 16), len + (size_t)k * npk, q + (size_t)k * npk, h + (size_t)k * npk, npk); }, reps));
    }
    return 0;
}
