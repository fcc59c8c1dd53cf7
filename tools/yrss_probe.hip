// yrss_probe.hip — measurement helper (not part of the product ABI).
//
// "Ideal traffic twin" of yrss_parse_hash: moves exactly the same bytes per
// packet (64-byte window + 2-byte data_len read, 2-byte queue + 4-byte hash
// written) in the same access layout as the parse kernel, with no parse work:
//   - 4-tile chunks dealt round-robin to 8 waves per CU (compact read window);
//   - each tile's four 16-byte non-temporal loads in flight while the previous
//     tile is handled (one tile ahead);
//   - the window reaches its packet's lane through LDS;
//   - outputs buffered in LDS and written per chunk as one burst of 16-byte
//     stores (1 KiB of hash, 512 B of q per wave-instruction), the parse
//     kernel's form; loads run one tile ahead across chunk boundaries too.
// Its duration on a given box is the practical floor for the parse kernel's
// traffic there; bench.py reports the parse kernel against it next to the
// 8 TB/s spec peak, so box-to-box HBM variance is visible.
// YRSS_PROBE_MODE=1 keeps only the reads (66 B/pkt), =2 only the writes
// (6 B/pkt), =3 only the writes as 16-byte stores: tools/probe_split.py
// compares their sum with the mixed run.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr uint32_t kC = 4;        // tiles per chunk
constexpr uint32_t kWaves = 8;    // per workgroup (512 threads), one workgroup per CU

template <int kMode>   // 0: reads + writes, 1: reads only, 2: writes only
__global__ __launch_bounds__(512) void yrss_probe_traffic(const u32x4 *win, const uint16_t *len,
                                                          int16_t *q, uint32_t *hash, uint32_t n)
{
    __shared__ u32x4 st[kWaves][256];
    __shared__ __attribute__((aligned(16))) uint32_t hb[kWaves][kC * 64];
    __shared__ __attribute__((aligned(16))) uint16_t qb[kWaves][kC * 64];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t W = gridDim.x * kWaves;
    const uint32_t gw = blockIdx.x * kWaves + w;
    const uint32_t ntiles = (n + 63u) / 64u;
    const uint32_t nchunk = (ntiles + kC - 1) / kC;
    u32x4 nx[4];
    uint16_t nl = 0;
    auto issue = [&](uint32_t t0) {
        if (kMode >= 2) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                nx[k] = u32x4{t0, lane, (uint32_t)k, n};
            nl = (uint16_t)t0;
            return;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = t0 + 16u * k + (lane >> 2);
            nx[k] = __builtin_nontemporal_load(win + (size_t)min(p, n - 1u) * 4u + (lane & 3u));
        }
        nl = len[min(t0 + lane, n - 1u)];
    };
    // the wave's tiles form one sequence across its chunks (as in the parse
    // kernel), loaded one tile ahead across chunk boundaries too
    auto tile_of = [&](uint32_t i) -> uint32_t {   // ntiles when past the wave's last
        const uint32_t c = gw + (i / kC) * W;
        if (c >= nchunk)
            return ntiles;
        const uint32_t t = c * kC + i % kC;
        return t < ntiles ? t : ntiles;
    };
    uint32_t seq = 0;
    if (tile_of(0) < ntiles)
        issue(tile_of(0) * 64u);
    for (uint32_t c = gw; c < nchunk; c += W) {
        const uint32_t tb = c * kC, te = min(tb + kC, ntiles);
        for (uint32_t t = tb; t < te; ++t, ++seq) {
            u32x4 cur[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                cur[k] = nx[k];
            const uint16_t cl = nl;
            const uint32_t tn = tile_of(seq + 1);
            if (tn < ntiles)
                issue(tn * 64u);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                st[w][(16u * k + (lane >> 2)) * 4u + (lane & 3u)] = cur[k];
            __builtin_amdgcn_wave_barrier();
            const u32x4 a = st[w][lane * 4u + 0], b = st[w][lane * 4u + 1];
            const u32x4 cc = st[w][lane * 4u + 2], d = st[w][lane * 4u + 3];
            __builtin_amdgcn_wave_barrier();
            const uint32_t x = a.x ^ b.y ^ cc.z ^ d.w ^ cl;
            hb[w][(t - tb) * 64u + lane] = x;
            qb[w][(t - tb) * 64u + lane] = (uint16_t)(x & 0x7fffu);
        }
        const uint32_t base = tb * 64u;
        if ((kMode == 3 || kMode == 0) && te - tb == kC) {   // 16 bytes per lane per store, as the parse kernel's bursts
            __builtin_amdgcn_wave_barrier();
            // write-through (sc1) 16-byte stores, exactly the parse kernel's burst form
            const __amdgpu_buffer_rsrc_t rh =
                __builtin_amdgcn_make_buffer_rsrc(hash + base, 0, (int)(kC * 64u * 4u), 0x00020000);
            const __amdgpu_buffer_rsrc_t rq =
                __builtin_amdgcn_make_buffer_rsrc(q + base, 0, (int)(kC * 64u * 2u), 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(reinterpret_cast<const u32x4 *>(hb[w])[lane], rh,
                                                   (int)(lane * 16u), 0, 16);
            if (lane < 32)
                __builtin_amdgcn_raw_buffer_store_b128(reinterpret_cast<const u32x4 *>(qb[w])[lane], rq,
                                                       (int)(lane * 16u), 0, 16);
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        if (kMode == 5) {   // outputs into the packets' own window records (DRAM-row locality test)
            for (uint32_t j = 0; j < te - tb; ++j) {
                const uint32_t e = j * 64u + lane;
                if (base + e < n) {
                    uint32_t *r = const_cast<uint32_t *>(reinterpret_cast<const uint32_t *>(win + (size_t)(base + e) * 4u));
                    *reinterpret_cast<uint2 *>(r) = uint2{hb[w][e], (uint32_t)qb[w][e]};
                }
            }
            continue;
        }
        for (uint32_t j = 0; j < te - tb; ++j) {
            const uint32_t e = j * 64u + lane;
            if (kMode == 1 && hb[w][e] != 0x9e3779b9u)   // reads only: practically never stores
                continue;
            if (base + e < n) {
                hash[base + e] = hb[w][e];
                q[base + e] = (int16_t)qb[w][e];
            }
        }
    }
}

// Write-phase experiment: the same traffic as mode 0, but each wave keeps the
// outputs of up to `cap` chunks (kB max) in LDS and writes them only when its
// buffer is full or, with kClock, when the chip-wide 100 MHz clock
// (s_memrealtime) enters a new period of `period` ticks -- so every wave's
// writes land in the same short window and the memory controllers see write
// bursts between long read phases instead of a trickle of writes.
constexpr uint32_t kB = 4;
template <bool kClock>
__global__ __launch_bounds__(512) void yrss_probe_phase(const u32x4 *win, const uint16_t *len,
                                                        int16_t *q, uint32_t *hash, uint32_t n,
                                                        uint32_t period, uint32_t cap)
{
    __shared__ u32x4 st[kWaves][256];
    __shared__ __attribute__((aligned(16))) uint32_t hb[kWaves][kB * kC * 64];
    __shared__ __attribute__((aligned(16))) uint16_t qb[kWaves][kB * kC * 64];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t W = gridDim.x * kWaves;
    const uint32_t gw = blockIdx.x * kWaves + w;
    const uint32_t ntiles = (n + 63u) / 64u;
    const uint32_t nchunk = (ntiles + kC - 1) / kC;
    u32x4 nx[4];
    uint16_t nl = 0;
    auto issue = [&](uint32_t t0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = t0 + 16u * k + (lane >> 2);
            nx[k] = __builtin_nontemporal_load(win + (size_t)min(p, n - 1u) * 4u + (lane & 3u));
        }
        nl = len[min(t0 + lane, n - 1u)];
    };
    uint32_t first = 0, np = 0;   // buffered chunks: first, first + W, ... (np of them)
    uint64_t last = kClock ? __builtin_amdgcn_s_memrealtime() / period : 0;
    auto flush = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t i = 0; i < np; ++i) {
            const uint32_t base = (first + i * W) * kC * 64u;
            const uint32_t cnt = min(kC * 64u, n - base);
            const uint32_t *h = hb[w] + i * kC * 64u;
            const uint16_t *qq = qb[w] + i * kC * 64u;
            if (cnt == kC * 64u) {
                reinterpret_cast<u32x4 *>(hash + base)[lane] = reinterpret_cast<const u32x4 *>(h)[lane];
                if (lane < 32)
                    reinterpret_cast<u32x4 *>(q + base)[lane] = reinterpret_cast<const u32x4 *>(qq)[lane];
            } else {
                for (uint32_t e = lane; e < cnt; e += 64u) {
                    hash[base + e] = h[e];
                    q[base + e] = (int16_t)qq[e];
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        np = 0;
    };
    for (uint32_t c = gw; c < nchunk; c += W) {
        const uint32_t tb = c * kC, te = min(tb + kC, ntiles);
        if (np == 0)
            first = c;
        issue(tb * 64u);
        for (uint32_t t = tb; t < te; ++t) {
            u32x4 cur[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                cur[k] = nx[k];
            const uint16_t cl = nl;
            if (t + 1 < te)
                issue((t + 1) * 64u);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                st[w][(16u * k + (lane >> 2)) * 4u + (lane & 3u)] = cur[k];
            __builtin_amdgcn_wave_barrier();
            const u32x4 a = st[w][lane * 4u + 0], b = st[w][lane * 4u + 1];
            const u32x4 cc = st[w][lane * 4u + 2], d = st[w][lane * 4u + 3];
            __builtin_amdgcn_wave_barrier();
            const uint32_t x = a.x ^ b.y ^ cc.z ^ d.w ^ cl;
            hb[w][np * kC * 64u + (t - tb) * 64u + lane] = x;
            qb[w][np * kC * 64u + (t - tb) * 64u + lane] = (uint16_t)(x & 0x7fffu);
        }
        ++np;
        bool due = np >= cap;
        if (kClock) {
            const uint64_t now = __builtin_amdgcn_s_memrealtime() / period;
            if (now != last) {
                due = true;
                last = now;
            }
        }
        if (due)
            flush();
    }
    flush();
}

}  // namespace

extern "C" int yrss_probe_phase_launch(const void *win, const void *len, void *q, void *hash,
                                       uint32_t npkts, void *stream, int clock, uint32_t period,
                                       uint32_t cap)
{
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return -5;
    if (npkts == 0)
        return 0;
    cap = cap < 1 ? 1 : (cap > kB ? kB : cap);
    period = period < 1 ? 1 : period;
    auto k = clock ? yrss_probe_phase<true> : yrss_probe_phase<false>;
    hipLaunchKernelGGL(k, dim3((unsigned)cus), dim3(512), 0, (hipStream_t)stream,
                       (const u32x4 *)win, (const uint16_t *)len, (int16_t *)q, (uint32_t *)hash,
                       npkts, period, cap);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int yrss_probe_traffic_launch_mode(const void *win, const void *len, void *q,
                                              void *hash, uint32_t npkts, void *stream, int mode);

extern "C" int yrss_probe_traffic_launch(const void *win, const void *len, void *q, void *hash,
                                         uint32_t npkts, void *stream)
{
    static int mode = -1;
    if (mode < 0) {
        const char *e = getenv("YRSS_PROBE_MODE");
        mode = e ? atoi(e) : 0;
    }
    return yrss_probe_traffic_launch_mode(win, len, q, hash, npkts, stream, mode);
}

// mode 0: the parse kernel's reads and writes; 1: its reads only; 2: its
// writes only; 3: see yrss_probe_traffic; 5: the same writes into the packets'
// own window records (8 bytes at the start of each), not separate arrays
extern "C" int yrss_probe_traffic_launch_mode(const void *win, const void *len, void *q,
                                              void *hash, uint32_t npkts, void *stream, int mode)
{
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return -5;
    }
    if (npkts == 0)
        return 0;
    auto k = mode == 1   ? yrss_probe_traffic<1>
             : mode == 2 ? yrss_probe_traffic<2>
             : mode == 3 ? yrss_probe_traffic<3>
             : mode == 5 ? yrss_probe_traffic<5>
                         : yrss_probe_traffic<0>;
    hipLaunchKernelGGL(k, dim3((unsigned)cus), dim3(512), 0, (hipStream_t)stream,
                       (const u32x4 *)win, (const uint16_t *)len, (int16_t *)q, (uint32_t *)hash,
                       npkts);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
