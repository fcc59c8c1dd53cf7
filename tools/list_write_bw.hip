// list_write_bw.hip — the write pattern of the line scatter's copy-out alone,
// with no ranks, no stage and no layout: how fast can 2^24 packet indices be
// written into nb per-bucket lists when each workgroup writes, span after
// span, one run of S/nb words into every list?  Separates the list-store
// pattern's own cost from the kernel's phase work.
//
//   list_write_bw N NB SPAN WG_PER_CU [AUX] [REPS]
//     N       packets (words of lists), a multiple of SPAN
//     NB      lists (buckets), SPAN % (16 NB) == 0: whole lines per run
//     SPAN    packets per span (8192, 16384)
//     WG_PER_CU  1 or 2: resident 512-thread workgroups per CU (LDS padding)
//     AUX     store cache policy: 2 nt (past 64 buckets), 18 nt|sc1, 0 plain
//     RD      0: writes only; 1: each span first reads 4 B a packet (two
//             16-bit streams, as the scatter's rank and q at > 128 buckets),
//             waits, then writes; 2: span g + 1's reads issued before span
//             g's writes (one span of look-ahead)
// Prints one JSON line: kernel us (mean of REPS), GB/s of list bytes.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kRsrcWord3 = 0x00020000;

template <int kAux, int kRd>
__global__ __launch_bounds__(512) void list_writes(uint32_t *lists, const uint16_t *ra,
                                                   const uint16_t *qa, uint32_t n, uint32_t nb,
                                                   uint32_t span, uint32_t xcd)
{
    extern __shared__ uint32_t pad[];
    const uint32_t t = threadIdx.x;
    const uint32_t nsp = n / span, G = gridDim.x;
    // workgroups of one XCD take consecutive ranges (as the line scatter)
    uint32_t r = blockIdx.x;
    if (xcd && G % 8u == 0)
        r = (blockIdx.x % 8u) * (G / 8u) + blockIdx.x / 8u;
    const uint32_t g0 = (uint32_t)((uint64_t)r * nsp / G), g1 = (uint32_t)((uint64_t)(r + 1) * nsp / G);
    const uint32_t run = span / nb;          // words per list per span
    const uint32_t len = n / nb;             // words per list
    const uint32_t qpr = run / 4u;           // quads per run
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(lists, 0, (int)(n * 4u),
                                                                        kRsrcWord3);
    if (t == 0)
        pad[0] = g0;   // keep the LDS allocation
    // the span's streams: span / 512 packets a thread, 16 bytes = 8 packets a load
    const uint32_t per = span / 512u / 8u;   // loads a thread per stream (<= 8)
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(ra), 0, (int)(n * 2u), kRsrcWord3);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(qa), 0, (int)(n * 2u), kRsrcWord3);
    u32x4 a[8], b[8];
    uint32_t acc = 0;
    auto load = [&](uint32_t g) {
#pragma unroll
        for (uint32_t k = 0; k < 8u; ++k)
            if (k < per) {
                const int off = (int)((g * span + 8u * (k * 512u + t)) * 2u);
                a[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 2));
                b[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rq, off, 0, 2));
            }
    };
    if (kRd == 2 && g0 < g1)
        load(g0);
    for (uint32_t g = g0; g < g1; ++g) {
        if (kRd == 1)
            load(g);
        if (kRd) {
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
#pragma unroll
            for (uint32_t k = 0; k < 8u; ++k)
                if (k < per)
                    acc += a[k].x ^ b[k].w;
        }
        if (kRd == 2 && g + 1u < g1)
            load(g + 1u);
        for (uint32_t v = t; v < span / 4u; v += 512u) {
            const uint32_t b = v / qpr, k = v - b * qpr;
            const uint32_t d = b * len + g * run + 4u * k;
            const uint32_t x = g * span + 4u * v + (acc & 0x80000000u);   // (keep the loads)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{x, x + 1u, x + 2u, x + 3u}, rs,
                                                   (int)(d * 4u), 0, kAux);
        }
        __syncthreads();
    }
}

int main(int argc, char **argv)
{
    if (argc < 5) {
        fprintf(stderr, "usage: list_write_bw N NB SPAN WG_PER_CU [AUX] [REPS]\n");
        return 2;
    }
    const uint32_t n = (uint32_t)strtoul(argv[1], 0, 0), nb = (uint32_t)strtoul(argv[2], 0, 0);
    const uint32_t span = (uint32_t)strtoul(argv[3], 0, 0), wpc = (uint32_t)strtoul(argv[4], 0, 0);
    const int aux = argc > 5 ? atoi(argv[5]) : 2;
    const int reps = argc > 6 ? atoi(argv[6]) : 20;
    const int rd = argc > 7 ? atoi(argv[7]) : 0;
    if (!n || !nb || !span || n % span || span % (16u * nb) || (wpc != 1 && wpc != 2) ||
        span > 32768u || span % 4096u || rd < 0 || rd > 2) {
        fprintf(stderr, "bad shape\n");
        return 2;
    }
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess)
        return 1;
    uint32_t *lists = nullptr;
    uint16_t *ra = nullptr, *qa = nullptr;
    if (hipMalloc((void **)&lists, (size_t)n * 4u) != hipSuccess ||
        hipMalloc((void **)&ra, (size_t)n * 2u) != hipSuccess ||
        hipMalloc((void **)&qa, (size_t)n * 2u) != hipSuccess)
        return 1;
    if (hipMemset(ra, 0, (size_t)n * 2u) != hipSuccess || hipMemset(qa, 0, (size_t)n * 2u) != hipSuccess)
        return 1;
    const uint32_t cus = (uint32_t)p.multiProcessorCount;
    const uint32_t grid = std::min<uint32_t>(cus * wpc, n / span);
    const size_t lds = wpc == 1 ? 100u * 1024u : 70u * 1024u;   // 1 or 2 resident per CU
    auto launch = [&](hipStream_t s) {
#define LW(A, R) hipLaunchKernelGGL((list_writes<A, R>), dim3(grid), dim3(512), lds, s, lists, ra, qa, n, \
                                     nb, span, 1u)
        if (aux == 18) {
            if (rd == 0) LW(18, 0); else if (rd == 1) LW(18, 1); else LW(18, 2);
        } else if (aux == 0) {
            if (rd == 0) LW(0, 0); else if (rd == 1) LW(0, 1); else LW(0, 2);
        } else {
            if (rd == 0) LW(2, 0); else if (rd == 1) LW(2, 1); else LW(2, 2);
        }
#undef LW
    };
    for (int i = 0; i < 3; ++i)
        launch(0);
    if (hipDeviceSynchronize() != hipSuccess)
        return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    // back to back between two events: the events' own fences amortised
    float total = 0.f;
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i)
        launch(0);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&total, a, b);
    // check: every list word is its packet index somewhere (sum of 0..n-1)
    uint32_t *h = (uint32_t *)malloc((size_t)n * 4u);
    (void)hipMemcpy(h, lists, (size_t)n * 4u, hipMemcpyDeviceToHost);
    uint64_t sum = 0;
    for (uint32_t i = 0; i < n; ++i)
        sum += h[i];
    const bool ok = sum == (uint64_t)n * (n - 1u) / 2u;
    const double us = total / reps * 1e3;
    printf("{\"tool\": \"list_write_bw\", \"n\": %u, \"nb\": %u, \"span\": %u, \"wg_per_cu\": %u, "
           "\"grid\": %u, \"aux\": %d, \"rd\": %d, \"us\": %.2f, \"GBps\": %.1f, \"sum_ok\": %s}\n",
           n, nb, span, wpc, grid, aux, rd, us, (double)n * (rd ? 8.0 : 4.0) / us / 1e3,
           ok ? "true" : "false");
    free(h);
    (void)hipFree(lists);
    (void)hipFree(ra);
    (void)hipFree(qa);
    return ok ? 0 : 1;
}
