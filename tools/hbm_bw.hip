// hbm_bw.hip — measurement helper (not part of the product): what streaming
// shapes reach on this box's HBM, to set the parse kernel's practical floor.
//
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_bw.hip -o tools/hbm_bw && tools/hbm_bw [MiB]
//
// Every variant moves the parse kernel's bytes for n packets: a 64-byte window
// per packet read (packed, stride 64), plus — for the "pkt" variants — 2-byte
// data_len read and 2-byte queue + 4-byte hash written, one lane per packet.
// Prints one JSON line per variant: µs per launch and GB/s of algorithmic bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
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

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p)
{
    if (NT)
        return __builtin_nontemporal_load(p);
    return *p;
}

// read-only: grid-stride over 16-byte chunks, U independent loads per lane per step
template <bool NT, int U>
__global__ __launch_bounds__(512) void rd_stride(const u32x4 *a, size_t nchunks, uint32_t *sink)
{
    const size_t T = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t x = 0;
    for (; i + (U - 1) * T < nchunks; i += U * T) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = ld<NT>(a + i + u * T);
#pragma unroll
        for (int u = 0; u < U; ++u)
            x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < nchunks; i += T) {
        const u32x4 v = ld<NT>(a + i);
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x9E3779B9u)
        sink[0] = x;
}

// write-only: grid-stride 16-byte stores of an index pattern (the 1-bucket
// scatter's list run), U stores per lane per step
template <bool NT, int U>
__global__ __launch_bounds__(512) void wr_stride(u32x4 *b, size_t nchunks, uint32_t base)
{
    const size_t T = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * T < nchunks; i += U * T) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t x = base + 4u * (uint32_t)(i + u * T);
            const u32x4 v = {x, x + 1u, x + 2u, x + 3u};
            if (NT)
                __builtin_nontemporal_store(v, b + i + u * T);
            else
                b[i + u * T] = v;
        }
    }
    for (; i < nchunks; i += T) {
        const uint32_t x = base + 4u * (uint32_t)i;
        const u32x4 v = {x, x + 1u, x + 2u, x + 3u};
        if (NT)
            __builtin_nontemporal_store(v, b + i);
        else
            b[i] = v;
    }
}

// write-only, the scatter's shape: one wave per group of G 16-byte vectors
// (G = 1024: a 4096-packet group's list), 1 KiB per wave-instruction
template <int G>
__global__ __launch_bounds__(256) void wr_group(u32x4 *b, size_t nchunks, uint32_t base)
{
    const size_t w = (size_t)blockIdx.x * 4 + threadIdx.x / 64;
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t v = lane; v < G; v += 64) {
        const size_t i = w * G + v;
        if (i < nchunks) {
            const uint32_t x = base + 4u * (uint32_t)i;
            __builtin_nontemporal_store(u32x4{x, x + 1u, x + 2u, x + 3u}, b + i);
        }
    }
}

// copy: read 16 B, write 16 B (the guide's float4 copy)
template <bool NT>
__global__ __launch_bounds__(512) void copy_stride(const u32x4 *a, u32x4 *b, size_t nchunks)
{
    const size_t T = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nchunks; i += T) {
        const u32x4 v = ld<NT>(a + i);
        if (NT)
            __builtin_nontemporal_store(v, b + i);
        else
            b[i] = v;
    }
}

// packet shape, persistent waves, contiguous segment per wave.  Per 64-packet
// tile: 4 x 16-B loads per lane (lane l reads chunk l&3 of packet 16k + l/4, so
// each wave-instruction is 1 KiB contiguous), len per lane, then per lane
// (one packet each) q and hash stores of full-wave runs.  The window bytes reach
// the packet's lane through LDS like the parse kernel (no parse work).
template <bool NT, int PF>
__global__ __launch_bounds__(512) void pkt_seg(const u32x4 *win, const uint16_t *len, int16_t *q,
                                               uint32_t *hash, uint32_t n, uint32_t seg)
{
    __shared__ u32x4 st[8][256];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t gw = blockIdx.x * 8u + w;
    const uint32_t beg = min(gw * seg, n), end = min(beg + seg, n);
    u32x4 nx[4];
    uint16_t nl = 0;
    auto issue = [&](uint32_t t0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = t0 + 16u * k + (lane >> 2);
            nx[k] = ld<NT>(win + (size_t)min(p, n - 1u) * 4u + (lane & 3u));
        }
        nl = len[min(t0 + lane, n - 1u)];
    };
    if (beg < end)
        issue(beg);
    for (uint32_t t0 = beg; t0 < end; t0 += 64u) {
        u32x4 cur[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            cur[k] = nx[k];
        }
        uint16_t cl = nl;
        if (PF && t0 + 64u < end)
            issue(t0 + 64u);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            st[w][(16u * k + (lane >> 2)) * 4u + (lane & 3u)] = cur[k];
        __builtin_amdgcn_wave_barrier();
        const u32x4 a = st[w][lane * 4u + 0], b = st[w][lane * 4u + 1];
        const u32x4 c = st[w][lane * 4u + 2], d = st[w][lane * 4u + 3];
        __builtin_amdgcn_wave_barrier();
        const uint32_t x = a.x ^ b.y ^ c.z ^ d.w ^ cl;
        const uint32_t p = t0 + lane;
        if (p < end) {
            __builtin_nontemporal_store((int16_t)(x & 0x7fff), q + p);
            __builtin_nontemporal_store(x, hash + p);
        }
        if (!PF && t0 + 64u < end)
            issue(t0 + 64u);
    }
}

// packet shape, chunk-interleaved: wave gw takes chunks gw, gw + W, gw + 2W, ...
// of C tiles (64 packets each), so the chip's concurrent reads form a sliding
// window of W*C tiles instead of W far-apart streams.  ST: 0 no stores, 1 per
// tile nt (2-B q / 4-B hash per lane), 2 per tile default policy, 3 per chunk
// batched through LDS into 16-B-per-lane stores (nt), 4 batched default.
template <int C, int PF, int ST = 1, int LN = 1>
__global__ __launch_bounds__(512) void pkt_chunk(const u32x4 *win, const uint16_t *len, int16_t *q,
                                                 uint32_t *hash, uint32_t n)
{
    __shared__ u32x4 st[8][256];
    __shared__ uint32_t hb[8][C * 64];
    __shared__ uint16_t qb[8][C * 64];
    const uint32_t lane = threadIdx.x & 63u, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t W = gridDim.x * 8u;
    const uint32_t gw = blockIdx.x * 8u + w;
    const uint32_t ntiles = (n + 63u) / 64u;
    const uint32_t nchunk = (ntiles + C - 1) / C;
    u32x4 nx[4];
    uint16_t nl = 0;
    auto issue = [&](uint32_t t0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = t0 + 16u * k + (lane >> 2);
            nx[k] = __builtin_nontemporal_load(win + (size_t)min(p, n - 1u) * 4u + (lane & 3u));
        }
        if (LN)
            nl = len[min(t0 + lane, n - 1u)];
    };
    for (uint32_t c = gw; c < nchunk; c += W) {
        const uint32_t tb = c * C, te = min(tb + C, ntiles);
        if (PF)
            issue(tb * 64u);
        for (uint32_t t = tb; t < te; ++t) {
            const uint32_t t0 = t * 64u;
            if (!PF)
                issue(t0);
            u32x4 cur[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                cur[k] = nx[k];
            const uint16_t cl = nl;
            if (PF && t + 1 < te)
                issue(t0 + 64u);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                st[w][(16u * k + (lane >> 2)) * 4u + (lane & 3u)] = cur[k];
            __builtin_amdgcn_wave_barrier();
            const u32x4 a = st[w][lane * 4u + 0], b = st[w][lane * 4u + 1];
            const u32x4 cc = st[w][lane * 4u + 2], d = st[w][lane * 4u + 3];
            __builtin_amdgcn_wave_barrier();
            const uint32_t x = a.x ^ b.y ^ cc.z ^ d.w ^ cl;
            const uint32_t p = t0 + lane;
            if (ST == 1) {
                if (p < n) {
                    __builtin_nontemporal_store((int16_t)(x & 0x7fff), q + p);
                    __builtin_nontemporal_store(x, hash + p);
                }
            } else if (ST == 2) {
                if (p < n) {
                    q[p] = (int16_t)(x & 0x7fff);
                    hash[p] = x;
                }
            } else if (ST >= 3) {
                hb[w][(t - tb) * 64u + lane] = x;
                qb[w][(t - tb) * 64u + lane] = (uint16_t)(x & 0x7fff);
            } else if (x == 0x9E3779B9u) {
                hash[0] = x;
            }
        }
        if (ST == 5 || ST == 6) {
            // batched at chunk end, but lane-granular stores (256 B / 128 B per instr)
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            const uint32_t base = tb * 64u;
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t e = k * 64u + lane;
                if (base + e < n) {
                    if (ST == 5) {
                        __builtin_nontemporal_store(hb[w][e], hash + base + e);
                        __builtin_nontemporal_store((int16_t)qb[w][e], q + base + e);
                    } else {
                        hash[base + e] = hb[w][e];
                        q[base + e] = (int16_t)qb[w][e];
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        } else if (ST >= 3) {
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            const uint32_t base = tb * 64u;          // chunk's first packet (full chunks here)
#pragma unroll
            for (int k = 0; k < C / 4; ++k) {        // hash: C*64*4 B = C KiB, 1 KiB per instr
                const uint32_t e = (k * 64u + lane) * 4u;
                const u32x4 v = *reinterpret_cast<const u32x4 *>(&hb[w][e]);
                if (base + e + 3u < n) {
                    if (ST == 3)
                        __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(hash + base + e));
                    else
                        *reinterpret_cast<u32x4 *>(hash + base + e) = v;
                }
            }
#pragma unroll
            for (int k = 0; k < (C + 7) / 8; ++k) {  // q: C*64*2 B, 1 KiB per instr
                const uint32_t e = (k * 64u + lane) * 8u;
                if (e < C * 64u) {
                    const u32x4 v = *reinterpret_cast<const u32x4 *>(&qb[w][e]);
                    if (base + e + 7u < n) {
                        if (ST == 3)
                            __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(q + base + e));
                        else
                            *reinterpret_cast<u32x4 *>(q + base + e) = v;
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
    }
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
};

template <typename F>
static float time_us(F f, int reps)
{
    Timer t;
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(t.a, 0));
    for (int r = 0; r < reps; ++r)
        f();
    CK(hipEventRecord(t.b, 0));
    CK(hipEventSynchronize(t.b));
    float ms;
    CK(hipEventElapsedTime(&ms, t.a, t.b));
    return ms * 1000.f / reps;
}

int main(int argc, char **argv)
{
    const size_t mib = argc > 1 ? strtoul(argv[1], 0, 10) : 1024;
    const size_t bytes = mib << 20;
    const size_t nchunks = bytes / 16;
    const uint32_t npk = (uint32_t)(bytes / 64);
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    u32x4 *a, *b;
    uint16_t *len;
    int16_t *q;
    uint32_t *h, *sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&len, npk * 2ull));
    CK(hipMalloc(&q, npk * 2ull));
    CK(hipMalloc(&h, npk * 4ull));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(len, 0, npk * 2ull));
    const int reps = 20;
    auto rep = [&](const char *name, double algo_bytes, float us) {
        printf("{\"variant\": \"%s\", \"us\": %.2f, \"GBps\": %.1f, \"bytes\": %.0f}\n", name, us,
               algo_bytes / us / 1e3, algo_bytes);
        fflush(stdout);
    };
    if (argc > 2 && !strcmp(argv[2], "write")) {
        // 4 rotating buffers of `sz` bytes (as the bench's 4 batches' lists)
        for (size_t sz : {(size_t)64 << 20, bytes / 4}) {
            const size_t nc = sz / 16;
            int r = 0;
            char nm[96];
#define W(NT, U, grid, label)                                                                     \
            snprintf(nm, sizeof nm, "write %s %zu MiB x4 rot", label, sz >> 20);                  \
            rep(nm, (double)sz, time_us([&] { wr_stride<NT, U><<<(grid), 512>>>(b + (r++ % 4) * nc, nc, 7u); }, reps));
            W(true, 1, (unsigned)cus, "nt U1 grid=1xCU")
            W(true, 4, (unsigned)cus, "nt U4 grid=1xCU")
            W(true, 1, (unsigned)cus * 2, "nt U1 grid=2xCU")
            W(true, 1, (unsigned)cus * 4, "nt U1 grid=4xCU")
            W(true, 1, (unsigned)(nc / 512), "nt U1 oneshot")
            W(false, 1, (unsigned)cus, "dflt U1 grid=1xCU")
            W(false, 1, (unsigned)(nc / 512), "dflt U1 oneshot")
            W(true, 1, (unsigned)(nc / 2048), "nt U1 grid=n/4")
#undef W
            snprintf(nm, sizeof nm, "write nt wave-per-16KiB (scatter shape) %zu MiB x4 rot", sz >> 20);
            rep(nm, (double)sz, time_us([&] { wr_group<1024><<<(unsigned)((nc / 1024 + 3) / 4), 256>>>(b + (r++ % 4) * nc, nc, 7u); }, reps));
        }
        return 0;
    }
    rep("read nt U4 grid=1xCU", (double)bytes,
        time_us([&] { rd_stride<true, 4><<<cus, 512>>>(a, nchunks, sink); }, reps));
    rep("read nt U1 oneshot", (double)bytes,
        time_us([&] { rd_stride<true, 1><<<(unsigned)(nchunks / 512), 512>>>(a, nchunks, sink); }, reps));
    const double pb = 72.0 * npk;
    const double rb = 66.0 * npk;
    for (int wpc : {8}) {
        const unsigned blocks = (unsigned)cus * wpc / 8u;
        char nm[96];
#define V(CC, ST, label, by)                                                                      \
        snprintf(nm, sizeof nm, "pkt C=%d %s wpc=%d", CC, label, wpc);                            \
        rep(nm, by, time_us([&] { pkt_chunk<CC, 1, ST, 1><<<blocks, 512>>>(a, len, q, h, npk); }, reps));
        V(4, 0, "nostore", rb)
        V(4, 1, "tile-nt", pb)
        V(4, 2, "tile-dflt", pb)
        V(4, 3, "chunk16B-nt", pb)
        V(4, 4, "chunk16B-dflt", pb)
        V(4, 5, "chunk4B-nt", pb)
        V(4, 6, "chunk4B-dflt", pb)
        V(4, 4, "chunk16B-dflt again", pb)
        V(16, 4, "chunk16B-dflt", pb)
        V(16, 6, "chunk4B-dflt", pb)
    }
    return 0;
}
