// yrss_probe.hip — measurement helper (not part of the product ABI).
//
// "Ideal traffic twin" of yrss_parse_hash: moves exactly the same bytes per
// packet (64-byte window + 2-byte data_len read, 2-byte queue + 4-byte hash
// written) with perfectly coalesced non-temporal 16-byte loads and no parse
// work.  Its duration on a given box is the practical floor for the parse
// kernel's traffic on that box; bench.py reports the parse kernel against it
// next to the 8 TB/s spec peak, so box-to-box HBM variance is visible.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void yrss_probe_traffic(const u32x4 *win, const uint16_t *len,
                                                          int16_t *q, uint32_t *hash,
                                                          uint32_t nchunks)
{
    const uint32_t i = blockIdx.x * 512u + threadIdx.x;   // one 16-byte chunk per lane
    if (i >= nchunks)
        return;
    const u32x4 v = __builtin_nontemporal_load(win + i);
    uint32_t x = v.x ^ v.y ^ v.z ^ v.w;
    x ^= __shfl_xor(x, 1, 64);
    x ^= __shfl_xor(x, 2, 64);
    if ((i & 3u) == 0u) {
        const uint32_t p = i >> 2;
        x ^= len[p];
        q[p] = (int16_t)(x & 0x7fffu);
        __builtin_nontemporal_store(x, hash + p);
    }
}

extern "C" int yrss_probe_traffic_launch(const void *win, const void *len, void *q, void *hash,
                                         uint32_t npkts, void *stream)
{
    const uint32_t nchunks = npkts * 4u;
    hipLaunchKernelGGL(yrss_probe_traffic, dim3((nchunks + 511u) / 512u), dim3(512), 0,
                       (hipStream_t)stream, (const u32x4 *)win, (const uint16_t *)len,
                       (int16_t *)q, (uint32_t *)hash, nchunks);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
