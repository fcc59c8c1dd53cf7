// yrss.hip — MI355X (gfx950) software-RSS engine: HIP kernels + the C ABI
// declared in include/yrss.h.
//
// Replaces, for a whole batch at once, the per-packet CPU path of yastack's
// F-Stack layer:
//   toeplitz_dispatch   fs/lib/ff_dpdk_if.c:1945-2113  (parse + queue)
//   toeplitz_hash       fs/lib/ff_dpdk_if.c:1881-1902  (bit-serial Toeplitz)
//   process_packets     fs/lib/ff_dpdk_if.c:1078-1094  (drop / enqueue to
//                                                        dispatch_ring[q])
//
// Three kernels per batch, all integer/byte work (no MFMA), HBM-bound:
//   1. yrss_parse_hash  one lane per packet.  A wave owns a contiguous segment
//      of packets and walks it in 64-packet tiles: four coalesced 16-byte
//      loads per lane bring the tile's 64-byte header windows in (1 KiB per
//      wave-instruction), they are staged through a wave-private 4 KiB LDS
//      tile in an XOR-swizzled packet-major layout, and each lane then reads
//      its own packet's fields back conflict-free.  The Toeplitz hash is 12
//      byte-table lookups in LDS (tables built per workgroup from the key
//      schedule); hash % nb_procs is a Lemire fastmod.  Writes q (int16) and
//      hash (u32); counts packets per bucket per wave segment with
//      ballot/readlane (one LDS update per distinct bucket per tile).
//   2. yrss_seg_scan    per bucket, exclusive scan of the segment counts.
//   3. yrss_scatter     each wave re-reads its segment's q (2 B/pkt) and writes
//      packet indices into the per-bucket lists with ballot ranks, in packet
//      order — the stable compaction that stands in for the FIFO
//      rte_ring_enqueue into dispatch_ring[port][q] (ff_dpdk_if.c:1087-1093).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <strings.h>
#include <time.h>

#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

#include "yrss.h"
#include "yrss_synth.h"
#ifdef YRSS_TEST_HOOKS
#include "yrss_test_hooks.h"
#endif

namespace {

constexpr int kWave = 64;
constexpr int kTile = 64;              // packets per wave-tile (one per lane)
constexpr int kScatterBlock = 256;     // 4 waves per scatter workgroup (halved for large nb)
constexpr int kScatterWaves = kScatterBlock / kWave;
constexpr uint32_t kMaxChunks = 65536;  // per launch; bounds the count matrix [nb][ncol]
constexpr uint32_t kLbMaxWgs = 2048;    // line-scatter ranges a range-bin row holds
constexpr uint32_t kCntWords = 2176;    // parse: per-wave LDS count slots (chunks x nb): 32 x 68
// scan: chunk columns per workgroup are up to kScanSub sub-tiles of 4096
// (ScanParams.sub): two where the columns come in whole 8192s, so a 65-bucket
// launch is 260 workgroups, resident at once, not 520 (scan 6.2 -> 5.3 us,
// profiles/r04_scan_subtile_ab.log); the column count stays a multiple of 4096
constexpr uint32_t kScanSub = 2;
constexpr uint32_t kScanTile = 4096;
constexpr uint32_t kPiece = 2048;       // fallback scatter: packets ranked and staged at once per wave
constexpr uint32_t kPieceSlots = kPiece / 64;   // 64-packet slots of a piece
// Toeplitz key tables: the 96 tuple bits are cut into 12 bytes (MSB first);
// table t maps a byte value to the XOR of the key windows its set bits select
// (12 lookups per hash).  Nibble tables (24 conflict-free lookups) and
// bit-serial VALU words were measured and gave nothing (profiles/r02_v1_*,
// r01_v29_*): the parse kernel is bound by its HBM stream, not the hash.
constexpr int kTblEntries = 256;
constexpr int kTblWordsPerTupleWord = 4 * kTblEntries;
constexpr int kTblWords = 3 * kTblWordsPerTupleWord;
constexpr int kTblBytes = kTblWords * 4;
constexpr int kRsrcWord3 = 0x00020000;  // buffer resource dword 3 for gfx9-family (CDNA)
constexpr uint32_t kOutTiles = 4;       // parse: output burst (tiles buffered in LDS)
constexpr int kOutBytes = kOutTiles * kTile * (4 + 2 + 1 + 2);   // hash, q, filter, rank
constexpr int kStageBytes = kTile * 64; // 4 KiB per wave

// Everything yrss_parse_hash needs, passed by value (kernarg segment).
struct ParseParams {
    const uint8_t *win;
    const uint16_t *len;
    int16_t *q;
    uint32_t *hash;       // may be null
    uint32_t *seg_cnt;    // [nb][ncol] per-chunk counts, bucket-major, or null
    uint16_t *rank;       // kCount == 2: packet's rank among its chunk's same-bucket packets
    uint32_t *fault;      // host-coherent fault record (report_fault), or null
    uint32_t n;
    uint32_t stride;
    uint32_t chunk;       // packets per chunk (dealt round-robin to waves), multiple of kTile
    uint32_t nchunk;      // chunks in this launch
    uint32_t ncol;        // row stride of seg_cnt (chunk columns, padded)
    uint32_t ct_shift;    // tiles per chunk = 2^ct_shift
    uint32_t nq;          // nb_queues
    uint32_t nb;          // buckets = nq + 1 (last = drop)
    uint32_t mod_d;       // divisor: nb_procs or nb_procs-1
    uint32_t q_off;       // 0 or 1 (dispatch_only_core)
    uint64_t mod_m;       // Lemire fastmod constant for mod_d
    int8_t *filter;       // protocol_filter class per packet, or null
    const uint32_t *kni_bm;   // tcp bitmap (2048 words) then udp bitmap (2048 words)
    uint32_t kni_enable;
    uint32_t out16;       // full output bursts as 16-byte write-through stores (0: lane-granular)
    uint32_t rank_pack;   // kCount == 2: the rank word is bucket << (ct_shift + 6) | rank
    uint32_t *tot_acc;    // kCount: per-bucket totals, added to (zeroed by the previous
                          // line scatter), or null (the scan kernel sums them)
    uint32_t *rbin;       // with tot_acc: [nb][kLbMaxWgs] counts per line-scatter range
    uint32_t rbin_chunks; // chunks a range (a multiple of 8)
    uint32_t kwin[96];    // key window at every tuple bit position
};

struct ScatterParams {
    const int16_t *q;
    const uint32_t *seg_off;   // [nb][ncol] exclusive per-bucket prefix per chunk
    const uint32_t *totals;    // [nb]
    uint32_t *qidx;
    uint32_t *qstart;          // [nb + 1]
    uint32_t *fault;           // host-coherent fault record
    uint32_t n;
    uint32_t seg;              // packets per span (one wave's unit: 2^gshift chunks)
    uint32_t nq;
    uint32_t nb;
    uint32_t nchunk;           // chunk columns written by the parse kernel
    uint32_t ncol;             // row stride of seg_off
    uint32_t gshift;           // a span is 2^gshift chunks
    uint32_t cshift;           // a chunk is 2^cshift packets
    uint32_t aux;              // words of a wave's per-bucket arrays ahead of its stage
    uint32_t stg;              // words of a wave's stage (kPiece + 3 per bucket, rounded)
    uint32_t wlds;             // words of LDS per wave
    uint32_t xcd;              // workgroups of one XCD take consecutive spans (xcd_block)
};

// Device-side fault record in host-coherent memory: {code, kernel, where,
// value}, the first fault of a batch wins (yrss_status / yrss_fault_info).
// Every guard on a rank-, count- or cursor-driven index reports here instead
// of storing, so a disagreement can neither fault the GPU nor pass silently.
__device__ __forceinline__ void report_fault(uint32_t *rec, uint32_t code, uint32_t kernel,
                                          uint32_t where, uint32_t value)
{
    if (!rec)
        return;
    uint32_t expected = 0u;
    if (__hip_atomic_compare_exchange_strong(rec, &expected, code, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
        __hip_atomic_store(rec + 1, kernel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(rec + 2, where, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(rec + 3, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Workgroup b runs on XCD b mod 8, each XCD with its own L2.  With `on`, the
// workgroups of one XCD take one contiguous range of logical blocks (a
// bijection for any grid size), so the scatter groups that share a list
// line at a run boundary are written through the same L2, where the two
// partial writes merge into one line before it leaves for HBM.
__device__ __forceinline__ uint32_t xcd_block(uint32_t on)
{
    const uint32_t b = blockIdx.x, nb = gridDim.x;
    if (!on || nb < 16u)
        return b;
    const uint32_t per = nb >> 3, rem = nb & 7u, x = b & 7u;
    return x * per + min(x, rem) + (b >> 3);
}

// orders a wave's LDS accesses across lanes (all lanes of one wave)
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// x, hidden from the optimiser: per-lane offsets derived from it inside a loop
// are recomputed there (a few VALU) instead of hoisted out and spilled
__device__ __forceinline__ uint32_t opaque(uint32_t x)
{
    asm volatile("" : "+v"(x));
    return x;
}

__device__ __forceinline__ uint64_t lane_lt_mask(uint32_t lane)
{
    return lane == 0 ? 0ull : (~0ull >> (64u - lane));
}

// Lanes (among `valid` ones) whose bucket equals this lane's: ceil(log2 nb)
// ballots, each keeping the lanes that agree on one bit (match-any emulation).
__device__ __forceinline__ uint64_t peer_mask(uint32_t bkt, bool valid, uint32_t nb)
{
    uint64_t peers = __ballot(valid);
    const uint32_t kbits = 32u - __builtin_clz(nb - 1u);   // nb >= 2
    for (uint32_t i = 0; i < kbits; ++i) {
        const uint64_t bi = __ballot((bkt >> i) & 1u);
        peers &= ((bkt >> i) & 1u) ? bi : ~bi;
    }
    return peers;
}

__device__ __forceinline__ uint32_t bucket_of(int qv, uint32_t nq)
{
    return (qv >= 0 && (uint32_t)qv < nq) ? (uint32_t)qv : nq;
}

// ---------------------------------------------------------------------------
// Kernel 1: parse + Toeplitz hash + queue (+ protocol_filter), one lane per
// packet.
// ---------------------------------------------------------------------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kKniWords = 2 * 2048;   // two 8 KiB port bitmaps (ff_dpdk_kni.c:312-328)

// One 64-packet tile's global loads: four 16-byte chunks per lane (lane l gets
// chunk l&3 of packet t0 + 16k + l/4, i.e. 1 KiB contiguous per instruction at
// stride 64) plus the lane's own data_len.  Addresses are clamped to the last
// packet of the segment instead of branching, so every load always issues.
template <bool kNT>
__device__ __forceinline__ void load_tile(const ParseParams &P, uint32_t t0, uint32_t end,
                                          uint32_t lane, u32x4 (&r)[4], uint32_t &L)
{
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t pk = min(t0 + 16u * k + (lane >> 2), end - 1u);
        const u32x4 *src = reinterpret_cast<const u32x4 *>(P.win + (size_t)pk * P.stride +
                                                           (lane & 3u) * 16u);
        r[k] = kNT ? __builtin_nontemporal_load(src) : *src;
    }
    L = P.len[min(t0 + lane, end - 1u)];
}

// Byte k of this lane's window: from the staged LDS tile (k < 64), else from
// HBM (k < stride, rare), else unavailable (*trunc).
__device__ __forceinline__ uint32_t win_byte(const ParseParams &P, const uint32_t *mine,
                                             uint32_t rsw, uint32_t pkt, uint32_t k, bool *trunc)
{
    if (k < 64u) {
        const uint32_t j = k >> 2;
        return (mine[(((j >> 2) ^ rsw) << 2) | (j & 3u)] >> (8u * (k & 3u))) & 0xffu;
    }
    if (k < P.stride)
        return P.win[(size_t)pkt * P.stride + k];
    *trunc = true;
    return 0u;
}

// Toeplitz over one 32-bit tuple word (bit 31-k selects key window k): four
// lookups into byte tables tb[j*256 + v], v = byte j of the word from the top.
__device__ __forceinline__ uint32_t tz_lds(uint32_t w, const uint32_t *tb)
{
    return tb[(w >> 24) & 0xffu] ^ tb[256 + ((w >> 16) & 0xffu)] ^
           tb[512 + ((w >> 8) & 0xffu)] ^ tb[768 + (w & 0xffu)];
}

// Table t, value v: XOR of key windows kwin[8t + b] over v's set bits b (b = 0
// is v's most significant bit).  Threads tid, tid + nthr, ...
__device__ __forceinline__ void build_key_tables(uint32_t *tbl, const uint32_t *kwin,
                                                 uint32_t tid, uint32_t nthr)
{
    for (uint32_t e = tid; e < (uint32_t)kTblWords; e += nthr) {
        const uint32_t t = e >> 8, v = e & 0xffu;
        uint32_t acc = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b)
            acc ^= (v & (0x80u >> b)) ? kwin[8 * t + b] : 0u;
        tbl[e] = acc;
    }
}

// FilterReturn values (ff_dpdk_kni.h:34-38) plus the two boundary outcomes.
constexpr int kFilterUnknown = -1, kFilterArp = 1, kFilterKni = 2;
constexpr int kFilterTrunc = -2;   // header walk left the staged window
constexpr int kFilterLoop = -3;    // IPIP with IHL=0: the reference recurses forever

__device__ __forceinline__ int kni_port_class(const uint32_t *kni, uint32_t proto, uint32_t raw)
{
    // get_bitmap(hdr->dst_port): index = port as stored (network order read
    // little-endian), bit 0x80 >> (idx % 8) of byte idx / 8 (ff_dpdk_kni.c:51-96)
    const uint32_t base = proto == 6u ? 0u : 2048u;
    const uint32_t byte = (kni[base + (raw >> 5)] >> (8u * ((raw >> 3) & 3u))) & 0xffu;
    return (byte & (0x80u >> (raw & 7u))) ? kFilterKni : kFilterUnknown;
}

// Generic protocol_filter_ip walk (ff_dpdk_kni.c:255-283) from IPv4 header at
// byte o with `left` bytes remaining, recursing through IPIP.  Rare path.
__device__ int kni_walk(const ParseParams &P, const uint32_t *kni, const uint32_t *mine,
                        uint32_t rsw, uint32_t pkt, uint32_t o, uint32_t left)
{
    bool trunc = false;
    for (;;) {
        if (left < 20u)
            return kFilterUnknown;
        const uint32_t hl = (win_byte(P, mine, rsw, pkt, o, &trunc) & 0x0fu) << 2;
        if (trunc)
            return kFilterTrunc;
        if (left < hl)
            return kFilterUnknown;
        const uint32_t pr = win_byte(P, mine, rsw, pkt, o + 9u, &trunc);
        if (trunc)
            return kFilterTrunc;
        const uint32_t nx = o + hl, nl = left - hl;
        if (pr == 6u || pr == 17u) {
            if (nl < (pr == 6u ? 20u : 8u))
                return kFilterUnknown;
            const uint32_t lo = win_byte(P, mine, rsw, pkt, nx + 2u, &trunc);
            const uint32_t hi = win_byte(P, mine, rsw, pkt, nx + 3u, &trunc);
            if (trunc)
                return kFilterTrunc;
            return kni_port_class(kni, pr, lo | (hi << 8));
        }
        if (pr != 4u)
            return kFilterUnknown;
        if (hl == 0u)
            return kFilterLoop;
        o = nx;
        left = nl;
    }
}

// One tile's slot of the wave's output buffer (LDS).
struct OutSlot {
    uint16_t *q;
    uint32_t *h;
    int8_t *f;
    uint16_t *r;
};

// Writes kOutTiles (or fewer) buffered tiles starting at packet t_first,
// issued back to back.  Bursts at batch end ran 4-5 % faster than per-tile
// stores interleaved with the read stream (kernel 200 vs 209 us on one box;
// tools/hbm_bw.hip "chunk4B-dflt" vs "tile-nt"), and the default policy beat
// non-temporal (which also evicted q before the scatter re-reads it: scatter
// 21.6 vs 25.5 us).  A full batch goes out as 16-byte write-through (sc1)
// stores, 0.8 % faster than lane-granular plain stores and 1.8 % faster than
// 16-byte plain ones (profiles/r01_v13_ahead_out16_ab.log); the batch-end
// remainder keeps the lane-granular stores.
// Buffer resources sized to the valid bytes drop lanes past the end, so every
// store issues and the vmcnt bookkeeping stays exact.
template <bool kFilter, bool kRank = false>
__device__ __forceinline__ void flush_out(const ParseParams &P, const uint16_t *oq,
                                          const uint32_t *oh, const int8_t *of,
                                          const uint16_t *orank, uint32_t t_first,
                                          uint32_t ntiles, uint32_t lane)
{
    const uint32_t nv = min(ntiles * (uint32_t)kTile, P.n - t_first);
    const __amdgpu_buffer_rsrc_t rq =
        __builtin_amdgcn_make_buffer_rsrc(P.q + t_first, 0, (int)(nv * 2u), kRsrcWord3);
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
        P.hash ? (void *)(P.hash + t_first) : (void *)P.q, 0, P.hash ? (int)(nv * 4u) : 0,
        kRsrcWord3);
    constexpr bool kRankWide = true;
    const bool wide = P.out16 && nv == ntiles * (uint32_t)kTile;
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        kRank ? (void *)(P.rank + t_first) : (void *)P.q, 0, kRank ? (int)(nv * 2u) : 0,
        kRsrcWord3);
    if (wide) {
        // a whole batch of tiles: 16-byte write-through (sc1) stores, 1 KiB of
        // hash and 512 B of q (and of ranks) per wave-instruction at 4 tiles;
        // the lines leave L2 at once, none is left dirty at kernel end (plain
        // rank stores left 32 MB of dirty lines in L2, written back inside the
        // next parse kernel: +7 us there, r03 A/B)
        wave_lds_sync();
        const uint32_t nh = nv >> 2, nq8 = nv >> 3;
        const u32x4 vh = *reinterpret_cast<const u32x4 *>(oh + 4u * min(lane, nh - 1u));
        const u32x4 vq = *reinterpret_cast<const u32x4 *>(oq + 8u * min(lane, nq8 - 1u));
        if (lane < nh)
            __builtin_amdgcn_raw_buffer_store_b128(vh, rh, (int)(lane * 16u), 0, 16);
        if (lane < nq8)
            __builtin_amdgcn_raw_buffer_store_b128(vq, rq, (int)(lane * 16u), 0, 16);
        if (kRank && kRankWide) {
            const u32x4 vr = *reinterpret_cast<const u32x4 *>(orank + 8u * min(lane, nq8 - 1u));
            if (lane < nq8)
                __builtin_amdgcn_raw_buffer_store_b128(vr, rr, (int)(lane * 16u), 0, 16);
        }
        wave_lds_sync();
    } else {
        for (uint32_t j = 0; j < ntiles; ++j) {
            const uint32_t e = j * kTile + lane;
            __builtin_amdgcn_raw_buffer_store_b16(oq[e], rq, (int)(e * 2u), 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(oh[e], rh, (int)(e * 4u), 0, 0);
        }
    }
    if (kFilter) {
        const __amdgpu_buffer_rsrc_t rf =
            __builtin_amdgcn_make_buffer_rsrc(P.filter + t_first, 0, (int)nv, kRsrcWord3);
        for (uint32_t j = 0; j < ntiles; ++j) {
            const uint32_t e = j * kTile + lane;
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)of[e], rf, (int)e, 0, 0);
        }
    }
    if (kRank && !(wide && kRankWide)) {
        for (uint32_t j = 0; j < ntiles; ++j) {
            const uint32_t e = j * kTile + lane;
            __builtin_amdgcn_raw_buffer_store_b16(orank[e], rr, (int)(e * 2u), 0, 0);
        }
    }
}

template <int kCount, bool kFilter>
__device__ __forceinline__ void process_tile(const ParseParams &P, const uint32_t *tbl,
                                             const uint32_t *kni, u32x4 *stage, uint32_t *cnt,
                                             const OutSlot &ob, uint32_t t0, uint32_t end,
                                             uint32_t lane, const u32x4 (&r)[4], uint32_t Lraw)
{
    // Staging layout: chunk c (16 B) of tile packet p at slot p*4 + (c ^ ((p>>2)&3)).
    // Writes: lane l holds chunk l&3 of packet 16k + l/4, so (p>>2)&3 == (l>>4)&3.
    // Reads: packet p = l, swizzle (l>>2)&3.  Both sides are bank-conflict free
    // (ds_write_b128 8-lane groups cover 128 contiguous bytes; ds_read_b128
    // 16-lane groups hit 16 distinct 16-byte slots).
    const uint32_t wsw = (lane >> 4) & 3u;
    const uint32_t rsw = (lane >> 2) & 3u;
    const uint32_t *mine = reinterpret_cast<const uint32_t *>(stage + lane * 4);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        stage[(16u * k + (lane >> 2)) * 4u + ((lane & 3u) ^ wsw)] = r[k];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    const uint32_t pkt = t0 + lane;
    const bool valid = pkt < end;
    const uint32_t L = valid ? Lraw : 0u;
    const u32x4 c0 = stage[lane * 4 + (0u ^ rsw)];
    const u32x4 c1 = stage[lane * 4 + (1u ^ rsw)];
    const uint32_t d3 = c0.w;          // bytes 12..15: ether_type, ver/IHL
    const uint32_t d5 = c1.y;          // bytes 20..23: proto at 23
    const uint32_t d6 = c1.z;          // bytes 24..27: saddr[0..1] at 26,27
    const uint32_t d7 = c1.w;          // bytes 28..31: saddr[2..3], daddr[0..1]
    const uint32_t d8 = mine[((2u ^ rsw) << 2) | 0u];   // bytes 32..35
    const uint32_t ihl = (d3 >> 16) & 0xfu;
    const uint32_t ihl4 = ihl << 2;
    const uint32_t proto = d5 >> 24;
    // L4 ports at p = 14 + 4*IHL: dwords 3+IHL (bytes 2,3) and 4+IHL (bytes 0,1).
    // IHL <= 11 keeps them inside the staged 64 bytes; IHL >= 12 needs bytes
    // 64..77 and takes the rare slow paths below.
    const uint32_t j = 3u + ihl;
    const bool tail = j + 1u >= 16u;
    const uint32_t jj = tail ? 3u : j;
    const uint32_t pa = mine[(((jj >> 2) ^ rsw) << 2) | (jj & 3u)];
    const uint32_t pb = mine[((((jj + 1u) >> 2) ^ rsw) << 2) | ((jj + 1u) & 3u)];

    // toeplitz_dispatch's checks (ff_dpdk_if.c:1956-1986)
    const uint32_t et = ((d3 & 0xffu) << 8) | ((d3 >> 8) & 0xffu);
    const bool eth = valid && L >= 14u;
    const bool ip_ok = eth && et == 0x0800u && L - 14u >= 20u && L - 14u >= ihl4;
    int qv = YRSS_DEFAULT_Q;
    if (eth && (et == 0x0806u || et == 0x8035u))
        qv = 0;
    const bool hashed = ip_ok && (L - ihl4) >= 20u && proto == 6u;
    uint32_t h = 0;
    if (hashed) {
        // Tuple = LE image of ntohl(src), ntohl(dst), ntohs(sport), ntohs(dport)
        // (ff_dpdk_if.c:1994-2021).
        // Tuple words in key order: w0 = saddr, w1 = daddr, w2 = ports; bit 31-k of
        // wi selects key window 32i+k; each word is 4 byte-table lookups.
        const uint32_t w0 = __builtin_amdgcn_alignbit(d7, d6, 16);
        const uint32_t w1 = __builtin_amdgcn_alignbit(d8, d7, 16);
        const uint32_t w2 = (pa & 0xffff0000u) | (pb & 0xffffu);
        const uint32_t h_l3 = tz_lds(w0, tbl) ^ tz_lds(w1, tbl + kTblWordsPerTupleWord);
        h = h_l3 ^ tz_lds(w2, tbl + 2 * kTblWordsPerTupleWord);
        bool trunc = false;
        // Rare slow path, entered only by waves that hold such a packet, so its
        // global loads (and the vmcnt drain they imply) stay off the hot loop.
        if (__builtin_expect(tail, 0)) {
            if (18u + ihl4 <= P.stride) {
                const uint32_t *g =
                    reinterpret_cast<const uint32_t *>(P.win + (size_t)pkt * P.stride);
                const uint32_t ta = __builtin_nontemporal_load(g + j);
                const uint32_t tb = __builtin_nontemporal_load(g + j + 1u);
                h = h_l3 ^ tz_lds((ta & 0xffff0000u) | (tb & 0xffffu), tbl + 2 * kTblWordsPerTupleWord);
            } else {
                trunc = true;
            }
        }
        // hash % d exactly, then +q_off (:2031-2034): a mask when d is a power
        // of two (d = 2 at the reference's nb_procs 3 with dispatch_only_core;
        // the branch is uniform), else Lemire's fastmod with a 64-bit M.  The
        // mask saved the hashed parse kernel 1.3-2.9 us in four same-process
        // A/Bs (profiles/r06_parse_abl_*, r06_ab_c16_*)
        const uint32_t rem = (P.mod_d & (P.mod_d - 1u)) == 0u
                                 ? h & (P.mod_d - 1u)
                                 : (uint32_t)__umul64hi(P.mod_m * (uint64_t)h, (uint64_t)P.mod_d);
        qv = (int)(uint16_t)(rem + P.q_off);
        if (trunc) {
            qv = YRSS_Q_TRUNCATED;
            h = 0u;
        }
    }

    int fc = kFilterUnknown;
    if (kFilter) {
        // protocol_filter (ff_dpdk_if.c:976-996) + ff_kni_proto_filter
        // (ff_dpdk_kni.c:218-290): ARP, else (KNI on, IPv4) the dst port of the
        // first TCP/UDP header, recursing through IPIP.
        bool slow = false;
        if (eth && et == 0x0806u) {
            fc = kFilterArp;
        } else if (P.kni_enable && ip_ok) {
            const uint32_t nl = L - 14u - ihl4;
            if (proto == 6u || proto == 17u) {
                if (nl >= (proto == 6u ? 20u : 8u)) {
                    if (tail)
                        slow = true;
                    else
                        fc = kni_port_class(kni, proto, pb & 0xffffu);
                }
            } else if (proto == 4u) {
                slow = true;
            }
        }
        if (__builtin_expect(slow, 0))
            fc = kni_walk(P, kni, mine, rsw, pkt, 14u, L - 14u);
    }
    // the next tile's ds_writes must not overtake this tile's ds_reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();

    // outputs go to the wave's LDS out-buffer; flush_out() writes them in
    // bursts of up to kOutTiles tiles
    ob.q[lane] = (uint16_t)qv;
    ob.h[lane] = h;
    if (kFilter)
        ob.f[lane] = (int8_t)fc;

    if (kCount) {
        // per-bucket counts of this chunk: lanes sharing a bucket are found
        // with ceil(log2 nb) ballots (match-any by bit slices); the lowest
        // lane of each group adds the group size.  Cost is independent of how
        // many distinct buckets the tile holds.  kCount == 2 also keeps each
        // packet's rank among the chunk's (one-launch kernels: the tile's)
        // packets of its bucket: the leader's
        // atomic returns the count before the group (a wave's LDS atomics run
        // in issue order, so tiles stay in packet order) and each lane adds
        // its position inside the group.
        const uint32_t bkt = bucket_of(qv, P.nq);
        const uint64_t peers = peer_mask(bkt, valid, P.nb);
        const uint64_t lt = lane_lt_mask(lane);
        const bool leader = valid && (peers & lt) == 0;
        if (kCount == 2) {
            uint32_t before = 0;
            if (leader)
                before = atomicAdd(&cnt[bkt], (uint32_t)__popcll(peers));
            const int ll = peers ? __builtin_ctzll(peers) : (int)lane;
            const uint32_t tag = P.rank_pack ? bkt << (P.ct_shift + 6u) : 0u;
            ob.r[lane] = (uint16_t)(tag | (__shfl(before, ll, kWave) + (uint32_t)__popcll(peers & lt)));
        } else if (leader) {
            atomicAdd(&cnt[bkt], (uint32_t)__popcll(peers));
        }
    }
}

// ---------------------------------------------------------------------------
// Kernel 1 entry.
//   kCount   1: also count packets per bucket per chunk (per-queue lists on);
//            2: and write each packet's rank among its chunk's packets of its
//            bucket (the ranked scatter places packets by it)
//   kFilter  also classify protocol_filter / KNI (one byte per packet)
//   kBlock   workgroup size (256/512): waves per CU, one key table per group
// Window loads are non-temporal (streaming): ~25 % faster than default-policy
// loads (profiles/r01_v32_nt_ab.log).
// LDS: key tables 12 KiB | staging 4 KiB per wave | count slots 8 KiB per wave |
//      output buffer 2.25 KiB per wave | KNI bitmaps 16 KiB (kFilter only).
// ---------------------------------------------------------------------------
template <int kCount, bool kFilter, int kBlock>
__global__ __launch_bounds__(kBlock) void yrss_parse_hash(ParseParams P)
{
    constexpr int kWaves = kBlock / kWave;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t *tbl = reinterpret_cast<uint32_t *>(smem);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint32_t lane = lane_id();
    u32x4 *stage = reinterpret_cast<u32x4 *>(smem + kTblBytes + wave * kStageBytes);
    uint32_t *cnt_base =
        reinterpret_cast<uint32_t *>(smem + kTblBytes + kWaves * kStageBytes);
    uint32_t *cnt_w = cnt_base + wave * kCntWords;
    uint8_t *out_w = reinterpret_cast<uint8_t *>(cnt_base + kWaves * kCntWords) + wave * kOutBytes;
    uint32_t *oh = reinterpret_cast<uint32_t *>(out_w);
    uint16_t *oq = reinterpret_cast<uint16_t *>(out_w + kOutTiles * kTile * 4);
    int8_t *of = reinterpret_cast<int8_t *>(out_w + kOutTiles * kTile * 6);
    uint16_t *orank = reinterpret_cast<uint16_t *>(out_w + kOutTiles * kTile * 7);
    uint32_t *kni = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(cnt_base) +
                                                 kWaves * (kCntWords * 4 + kOutBytes));

    const uint32_t gw = blockIdx.x * kWaves + wave;
    const uint32_t W = gridDim.x * kWaves;

    build_key_tables(tbl, P.kwin, threadIdx.x, kBlock);
    if (kFilter)
        for (uint32_t e = threadIdx.x; e < (uint32_t)kKniWords; e += kBlock)
            kni[e] = P.kni_enable ? P.kni_bm[e] : 0u;
    if (kCount)
        for (uint32_t e = lane; e < kCntWords; e += kWave)
            cnt_w[e] = 0;
    __syncthreads();

    // Chunks are dealt round-robin (chunk c to wave c mod W), so at any moment
    // the chip reads a compact sliding window of the batch.  One contiguous
    // segment per wave had 4096 far-apart streams in flight and ran ~10 %
    // slower on the same box (tools/hbm_bw.hip: pkt_seg vs pkt_chunk).
    // Each chunk's per-bucket counts accumulate in its own LDS slot and are
    // stored once, after the last chunk: no global traffic but the windows and
    // the outputs inside the loop (a per-chunk flush sat in the in-order vmcnt
    // queue ahead of the next chunk's loads: +13 us on all-TCP).
    // The wave's tiles form one sequence across its chunks (chunk k is c =
    // gw + k*W; tile i is tile i mod 2^ct_shift of chunk i >> ct_shift), walked
    // with one tile of loads in flight ahead of the tile being parsed.  Two
    // register sets, unrolled by two, so no copy at the latch waits on a load;
    // the look-ahead load always issues (it re-reads the current tile at the
    // end) so the wait counts are the same on every path.
    // The host sizes chunks so a wave's slots fit (layout_for); a wave that
    // would own more chunks than it has slots reports and does nothing (the
    // check sits outside the loop: a fault-report branch inside it cost the
    // loop's load scheduling)
    bool slots_ok = true;   // (the wave still takes part in the workgroup's barriers)
    if (kCount) {
        const uint32_t own = P.nchunk > gw ? (P.nchunk - gw + W - 1u) / W : 0u;
        if (own * P.nb > kCntWords) {
            slots_ok = false;
            if (lane == 0)
                report_fault(P.fault, YRSS_FAULT_COUNT_SLOT, YRSS_K_PARSE_HASH, gw, own);
        }
    }
    auto tile_at = [&](uint32_t i, uint32_t &t0, uint32_t &slot) -> bool {
        const uint32_t kk = i >> P.ct_shift;
        const uint64_t c = gw + (uint64_t)kk * W;
        const uint64_t t = c * P.chunk + ((uint64_t)(i & ((1u << P.ct_shift) - 1u)) * kTile);
        if (c >= P.nchunk || t >= P.n)
            return false;
        t0 = (uint32_t)t;
        slot = kk;
        return true;
    };
    // outputs are buffered per batch of up to kOutTiles consecutive tiles of a
    // chunk and flushed after its last tile (or the sequence's last)
    const uint32_t fb_mask = (1u << min(P.ct_shift, 2u)) - 1u;   // kOutTiles = 4
    auto slot = [&](uint32_t i) {
        const uint32_t j = (i & fb_mask) * kTile;
        return OutSlot{oq + j, oh + j, of + j, orank + j};
    };
    auto after = [&](uint32_t i, uint32_t t0, bool last) {
        if (((i + 1u) & fb_mask) == 0u || last)
            flush_out<kFilter, kCount == 2>(P, oq, oh, of, orank, t0 - (i & fb_mask) * kTile,
                                            (i & fb_mask) + 1u, lane);
    };
    constexpr int kC = kCount;
    uint32_t tA = 0, sA = 0, tB = 0, sB = 0;
    if (slots_ok && tile_at(0, tA, sA)) {
        u32x4 rA[4], rB[4];
        uint32_t LA, LB;
        load_tile<true>(P, tA, P.n, lane, rA, LA);
        for (uint32_t i = 0;; i += 2) {
            const bool hB = tile_at(i + 1, tB, sB);
            load_tile<true>(P, hB ? tB : tA, P.n, lane, rB, LB);
            process_tile<kC, kFilter>(P, tbl, kni, stage, cnt_w + sA * P.nb, slot(i), tA, P.n,
                                      lane, rA, LA);
            after(i, tA, !hB);
            if (!hB)
                break;
            const bool hA = tile_at(i + 2, tA, sA);
            load_tile<true>(P, hA ? tA : tB, P.n, lane, rA, LA);
            process_tile<kC, kFilter>(P, tbl, kni, stage, cnt_w + sB * P.nb, slot(i + 1), tB,
                                      P.n, lane, rB, LB);
            after(i + 1, tB, !hA);
            if (!hA)
                break;
        }
    }
    if (kCount) {
        // Workgroup flush: for its j-th chunk each of the 8 waves owns column
        // blockIdx.x * 8 + w + j * W, so the workgroup's columns of round j
        // are 8 consecutive words of every bucket row.  Thread e takes wave
        // e % 8, bucket (e / 8) % nb, round e / (8 nb): a 64-lane store then
        // covers 8 rows x 32 contiguous bytes instead of one word in each of
        // 64 rows (a store costs the lines its lanes touch; the per-wave flush
        // it replaced cost 2 us on UDP and 33 us at 256 buckets,
        // profiles/r02_v30_cntwg_ab.log).
        __syncthreads();
        const uint32_t g0 = blockIdx.x * kWaves;
        const uint32_t kmax = P.nchunk > g0 ? (P.nchunk - g0 + W - 1) / W : 0u;
        // element e = (j * nb + b) * kWaves + w; the block size is a multiple
        // of kWaves, so a thread keeps its wave w and steps m = j * nb + b by
        // kBlock / kWaves, carried into (j, b) without a division.  The flush
        // costs ~5 us at 65 and 256 buckets, ~0 at 4 (a build without it,
        // profiles/r04_cntflush_ab.log).
        // Plain stores: written through (nt | sc1) the counts made the scan
        // reading them 1 us slower at 65 buckets, and the parse kernel was
        // -6 us in one run and +3 us in another (profiles/r04_flush_policy_ab.log,
        // r04_early_flush_ab.log)
        static_assert(kBlock % kWaves == 0, "a thread keeps its wave");
        // With tot_acc the workgroup also sums its counts per bucket (in the
        // staging LDS, free after the loop) and adds them to the batch totals,
        // so the line scatter needs no scan kernel in front of it
        // and, per round j, the 8 waves' counts of each bucket (their 8
        // consecutive columns g0 + j W + w lie in one scatter range: ranges
        // are multiples of 8 chunks and g0 of 8), added to that range's bin
        uint32_t *wtot = reinterpret_cast<uint32_t *>(smem + kTblBytes);
        uint32_t *jtot = wtot + P.nb;   // [kmax][nb] (kmax nb <= kCntWords)
        const bool tot = P.tot_acc != nullptr;   // (uniform)
        if (tot) {
            for (uint32_t e = threadIdx.x; e < P.nb * (kmax + 1u); e += kBlock)
                wtot[e] = 0u;
            __syncthreads();
        }
        const uint32_t w = threadIdx.x % kWaves;
        uint32_t j = 0, b = threadIdx.x / kWaves;
        while (b >= P.nb) {
            b -= P.nb;
            ++j;
        }
        while (j < kmax) {
            const uint32_t col = g0 + w + j * W;
            if (col < P.nchunk && (j + 1u) * P.nb <= kCntWords) {
                const uint32_t v = cnt_base[w * kCntWords + j * P.nb + b];
                P.seg_cnt[(size_t)b * P.ncol + col] = v;
                if (tot && v) {
                    atomicAdd(&wtot[b], v);
                    atomicAdd(&jtot[j * P.nb + b], v);
                }
            }
            b += kBlock / kWaves;
            while (b >= P.nb) {
                b -= P.nb;
                ++j;
            }
        }
        if (tot) {
            __syncthreads();
            for (uint32_t e = threadIdx.x; e < P.nb; e += kBlock)
                if (wtot[e])
                    __hip_atomic_fetch_add(P.tot_acc + e, wtot[e], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            for (uint32_t e = threadIdx.x; e < kmax * P.nb; e += kBlock) {
                const uint32_t jj = e / P.nb, bb = e - jj * P.nb;
                if (jtot[e])
                    __hip_atomic_fetch_add(P.rbin + bb * kLbMaxWgs + (g0 + jj * W) / P.rbin_chunks,
                                           jtot[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Kernel 2: per-bucket exclusive scan over the chunk columns, single pass.
// Workgroup (b, p) scans columns [p*4096, (p+1)*4096) of bucket row b (one
// uint4 per thread), publishes its tile total, and adds the totals of every
// earlier tile of the row, read at once by one lane each.  All counts exist
// when the kernel starts (the parse kernel wrote them), so every tile can
// publish at once and no tile waits on a chain of inclusive prefixes (a
// serial look-back over 16 tiles was most of this kernel's 5 us).  Status
// words carry the launch epoch, so they need no clearing between launches.
// The spin is bounded: a tile total that never appears sets *fault instead of
// hanging the GPU.
// ---------------------------------------------------------------------------
constexpr int kScanBlock = 1024;
static_assert(kMaxChunks / kScanTile <= kWave, "one look-back lane per scan tile");
static_assert(kScanBlock * 4 == 4096, "a sub-tile is one 16-byte word a thread");
constexpr uint64_t kStFlagP = 1ull << 63;   // status holds the inclusive prefix

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, uint32_t lane)
{
    // DPP: Hillis-Steele inside each 16-lane row (row_shr 1, 2, 4, 8), then
    // row 0's last lane into row 1, rows 0-1's into rows 2-3 (row_bcast 15,
    // 31 of the gfx9 DPP set): six VALU ops and no LDS round trip, where
    // shuffles cost a ds_bpermute and its wait per step
    (void)lane;
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);   // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return x;
}

struct ScanParams {
    const uint32_t *cnt;     // [nb][ncol]
    uint32_t *off;           // [nb][ncol] exclusive prefix per chunk column
    uint32_t *totals;        // [nb]
    unsigned long long *status;   // [nb][tiles]: flag | epoch:31 | value:32
    uint32_t *fault;
    uint32_t nchunk, ncol, tiles, epoch;
    uint32_t sub;            // 4096-column sub-tiles a workgroup (1..kScanSub)
};

__device__ __forceinline__ unsigned long long scan_status(uint32_t epoch, bool incl, uint32_t v)
{
    return (incl ? kStFlagP : 0ull) | ((unsigned long long)(epoch & 0x7fffffffu) << 32) | v;
}

__global__ __launch_bounds__(kScanBlock) void yrss_seg_scan(ScanParams P)
{
    // kScanSub sub-tiles of 4096 columns, sub-tile k's 16-byte word t at
    // column 4 (k 1024 + t): every load instruction reads 16 KB contiguous,
    // and each sub-tile is its own block scan, offset by the earlier ones
    __shared__ uint32_t wsum[kScanSub][kScanBlock / kWave];
    __shared__ uint32_t sub_sh[kScanSub];
    __shared__ uint32_t prefix_sh;
    const uint32_t b = blockIdx.x / P.tiles, p = blockIdx.x % P.tiles;
    const uint32_t lane = lane_id(), wave = threadIdx.x / kWave;
    const uint4 *row = reinterpret_cast<const uint4 *>(P.cnt + (size_t)b * P.ncol);
    uint4 v[kScanSub];
    uint32_t local[kScanSub], x[kScanSub];
#pragma unroll
    for (uint32_t k = 0; k < kScanSub; ++k) {
        const uint32_t col = (p * P.sub + k) * kScanTile + threadIdx.x * 4u;
        v[k] = k < P.sub ? row[col / 4u] : uint4{0u, 0u, 0u, 0u};
        // columns past the last chunk were never written this launch
        if (col + 0u >= P.nchunk) v[k].x = 0;
        if (col + 1u >= P.nchunk) v[k].y = 0;
        if (col + 2u >= P.nchunk) v[k].z = 0;
        if (col + 3u >= P.nchunk) v[k].w = 0;
        local[k] = v[k].x + v[k].y + v[k].z + v[k].w;
        x[k] = wave_incl_scan(local[k], lane);
        if (lane == kWave - 1)
            wsum[k][wave] = x[k];
    }
    __syncthreads();
    if (wave == 0) {
        uint32_t total = 0;
#pragma unroll
        for (uint32_t k = 0; k < kScanSub; ++k) {
            const uint32_t w = lane < kScanBlock / kWave ? wsum[k][lane] : 0u;
            const uint32_t ws = wave_incl_scan(w, lane);
            if (lane < kScanBlock / kWave)
                wsum[k][lane] = ws;
            if (lane == 0)
                sub_sh[k] = total;
            total += __shfl(ws, kScanBlock / kWave - 1, kWave);
        }
        // publish the tile total, then sum every predecessor's aggregate at
        // once (one lane per tile, <= 64 tiles per row), so no tile waits on
        // a chain of inclusive prefixes
        unsigned long long *st = P.status + (size_t)b * P.tiles;
        if (lane == 0)
            __hip_atomic_store(&st[p], scan_status(P.epoch, false, total), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        uint32_t mine = 0, spins = 0;
        bool ready = lane >= p;
        while (!__all(ready)) {
            if (!ready) {
                const unsigned long long w =
                    __hip_atomic_load(&st[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)((w >> 32) & 0x7fffffffu) == (P.epoch & 0x7fffffffu)) {
                    mine = (uint32_t)w;
                    ready = true;
                }
            }
            if (++spins > (1u << 22)) {
                if (lane == 0)
                    report_fault(P.fault, YRSS_FAULT_SCAN_TIMEOUT, YRSS_K_SCAN, b, p);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const uint32_t prefix = __shfl(wave_incl_scan(mine, lane), kWave - 1, kWave);
        if (lane == 0) {
            prefix_sh = prefix;
            if (p == P.tiles - 1)
                P.totals[b] = prefix + total;
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kScanSub; ++k) {
        if (k >= P.sub)
            break;
        const uint32_t col = (p * P.sub + k) * kScanTile + threadIdx.x * 4u;
        uint32_t run = prefix_sh + sub_sh[k] + x[k] - local[k] + (wave ? wsum[k][wave - 1] : 0u);
        uint4 o;
        o.x = run; run += v[k].x;
        o.y = run; run += v[k].y;
        o.z = run; run += v[k].z;
        o.w = run;
        reinterpret_cast<uint4 *>(P.off + (size_t)b * P.ncol)[col / 4u] = o;
    }
}

// List stores are streaming and written through at device scope (nt | sc1):
// with non-temporal stores alone the lines stayed dirty past the scatter and
// their write-back landed in the next batch's parse kernel (+19 us there at 9
// buckets, same-process A/B, profiles/r03_ab_inproc_store.log).
constexpr int kListAux = 18;   // nt | sc1
// Past 64 buckets the line scatter's stores are non-temporal only: its
// scatter ran 1.5-2.3 us (65 buckets) and 2.3-3.9 us (256) faster and the next
// batch's parse kernel no slower; at 9 buckets nt alone slowed the next parse
// kernel (+19 us in round 3, +7 in round 4), so fewer buckets keep nt | sc1
// (profiles/r04_list_policy_ab.log, r04_partial_quads_ab.log)
constexpr int kListAuxMany = 2;   // nt
constexpr uint32_t kListNtBuckets = 64;

// The lists as a buffer resource: offsets are 32-bit, so lists past 2^29
// entries take flat non-temporal stores instead (wide = false).
struct ListOut {
    __amdgpu_buffer_rsrc_t r;
    uint32_t *p;
    bool wide;
};
__device__ __forceinline__ ListOut list_out(uint32_t *qidx, uint32_t n)
{
    const bool wide = n < (1u << 29);
    return ListOut{__builtin_amdgcn_make_buffer_rsrc(qidx, 0, wide ? (int)(n * 4u) : 0, kRsrcWord3),
                   qidx, wide};
}
template <int kAux>
__device__ __forceinline__ void list_store4(const ListOut &o, uint32_t d, u32x4 v)
{
    if (o.wide)
        __builtin_amdgcn_raw_buffer_store_b128(v, o.r, (int)(d * 4u), 0, kAux);
    else
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(o.p + d));
}
template <int kAux>
__device__ __forceinline__ void list_store1(const ListOut &o, uint32_t d, uint32_t v)
{
    if (o.wide)
        __builtin_amdgcn_raw_buffer_store_b32(v, o.r, (int)(d * 4u), 0, kAux);
    else
        o.p[d] = v;
}

// The line scatter's lists: always one buffer resource (the host runs it on
// batches below kLineMaxPkts only, so n x 4 bytes fit the 32-bit record
// count and offsets), one store form a site: the flat fallback's second
// store at every site was a pair of branches a quad.
constexpr uint32_t kLineMaxPkts = 1u << 30;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t line_out(uint32_t *qidx, uint32_t n)
{
    return __builtin_amdgcn_make_buffer_rsrc(qidx, 0, (int)(n * 4u), kRsrcWord3);
}
template <int kAux>
__device__ __forceinline__ void line_store4(__amdgpu_buffer_rsrc_t r, uint32_t d, u32x4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(d * 4u), 0, kAux);
}
template <int kAux>
__device__ __forceinline__ void line_store1(__amdgpu_buffer_rsrc_t r, uint32_t d, uint32_t v)
{
    __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)(d * 4u), 0, kAux);
}

// ---------------------------------------------------------------------------
// Kernel 3b: the lists when a parse chunk is longer than the line scatter's
// span (batches past ~2^29 packets): the stable scatter of packet indices into
// the per-bucket lists, the FIFO rte_ring_enqueue into dispatch_ring[port][q]
// of process_packets (ff_dpdk_if.c:1087-1093), ranking from q itself.
//
// Persistent: as many waves as are resident, wave w taking spans w, w + W, ...
// (a span is 2^gshift parse chunks), so the waves in flight together cover one
// stretch of the batch.  A span's lists start at its buckets' prefixes from the
// scan (start[b] + prefix[b][first chunk]).  The span is worked in pieces of
// up to kPiece packets, each in three steps that touch only LDS and registers:
//   count  the piece's q (loaded slot-major, 32 x 64 packets, one piece ahead)
//          is histogrammed per bucket: lanes sharing a bucket are found with
//          ceil(log2 nb) ballots, the lowest adds the group's size;
//   place  every packet's stage slot is its bucket's run start + its rank:
//          the same ballots, and the leader's LDS atomic returns the count
//          before its group (a wave's LDS atomics run in issue order, so
//          slots, and therefore the lists, keep packet order);
//   copy   the stage is written out in order.  A bucket's run starts at a
//          stage slot congruent to its list position mod 4 (at most 3 words
//          of padding per bucket), so four stage words that share a bucket
//          are one aligned 16-byte store, the rest word by word.
// A span's histogram is checked against the parse kernel's counts at its end.
// Any disagreement, and any destination outside the batch, is reported
// through the fault record instead of stored (YRSS_FAULT_COUNT_MISMATCH /
// _LIST_RANGE / _STAGE).  Ranking in the scatter costs ~70 VALU per 64
// packets (ballots, twice), against ~13 for placing by the parse kernel's
// ranks, so this is the large-batch path only (yrss_scatter_lines otherwise).
// ---------------------------------------------------------------------------

// The piece's q (or ranks), slot-major (slot s, lane l -> packet p0 + 64 s +
// l), one register a slot: packing two slots per register at the load made
// every pair wait for its loads (and, behind them in the in-order vmcnt
// queue, for the previous piece's stores).  Lanes past the piece's end read 0
// through the buffer's range check and are masked by index.
__device__ __forceinline__ void load_piece(const uint16_t *q, uint32_t p0, uint32_t pe,
                                           uint32_t lane, uint32_t (&qv)[kPieceSlots])
{
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(q + p0), 0, (int)((pe - p0) * 2u), kRsrcWord3);
#pragma unroll
    for (uint32_t s = 0; s < kPieceSlots; ++s)
        qv[s] = __builtin_amdgcn_raw_buffer_load_b16(rq, (int)((s * 64u + lane) * 2u), 0,
                                                     2 /* nt */);
}

// Histogram (cnt) or placement (cur, stage) of one piece.  kPlace: each valid
// packet's stage word is (packet - p0) << 9 | bucket.
template <bool kPlace>
__device__ __forceinline__ void rank_piece(const ScatterParams &P,
                                           const uint32_t (&qv)[kPieceSlots], uint32_t p0,
                                           uint32_t pe, uint32_t lane_, uint32_t *ctr, uint32_t *stg)
{
    const uint32_t lane = opaque(lane_);
    const uint64_t lt = lane_lt_mask(lane);
    constexpr uint32_t kB = 8;   // slots whose LDS atomics issue back to back
#pragma unroll
    for (uint32_t s0 = 0; s0 < kPieceSlots; s0 += kB) {
        uint32_t bk[kB], first[kB];
        uint64_t peers[kB];
        bool valid[kB];
#pragma unroll
        for (uint32_t j = 0; j < kB; ++j) {
            const uint32_t s = s0 + j;
            const uint32_t p = p0 + s * 64u + lane;
            valid[j] = p < pe;
            bk[j] = bucket_of((int16_t)qv[s], P.nq);
            const uint32_t b0 = __builtin_amdgcn_readfirstlane(bk[j]);
            if (__all(valid[j] && bk[j] == b0))   // a whole slot of one bucket (UDP stretches)
                peers[j] = ~0ull;
            else
                peers[j] = peer_mask(bk[j], valid[j], P.nb);
        }
#pragma unroll
        for (uint32_t j = 0; j < kB; ++j) {
            first[j] = 0;
            if (valid[j] && (peers[j] & lt) == 0) {
                if (kPlace)
                    first[j] = atomicAdd(&ctr[bk[j]], (uint32_t)__popcll(peers[j]));
                else
                    atomicAdd(&ctr[bk[j]], (uint32_t)__popcll(peers[j]));
            }
        }
        if (kPlace) {
#pragma unroll
            for (uint32_t j = 0; j < kB; ++j) {
                const int leader = peers[j] ? __builtin_ctzll(peers[j]) : (int)lane;
                const uint32_t slot =
                    __shfl(first[j], leader, kWave) + (uint32_t)__popcll(peers[j] & lt);
                if (valid[j]) {
                    const uint32_t off = (s0 + j) * 64u + lane;
                    if (slot < P.stg)
                        stg[slot] = (off << 9) | bk[j];
                    else
                        report_fault(P.fault, YRSS_FAULT_STAGE, YRSS_K_SCATTER, p0 + off, slot);
                }
            }
        }
    }
}

// Writes a piece's stage out, quad by quad: four words of one bucket are one
// aligned 16-byte store (non-temporal when the piece writes the whole line),
// others word by word.  Returns how many entries this lane wrote.
__device__ __forceinline__ uint32_t copy_out(const ScatterParams &P, const uint32_t *stg,
                                             const uint32_t *base, const uint32_t *ls,
                                             const uint32_t *cnt, uint32_t p0, uint32_t ph,
                                             uint32_t lane)
{
    uint32_t wrote = 0;
    for (uint32_t v = lane; v < P.stg / 4u; v += kWave) {
        const u32x4 e = reinterpret_cast<const u32x4 *>(stg)[v];
        const uint32_t b = e.x & 511u;
        if (b < P.nb && (e.y & 511u) == b && (e.z & 511u) == b && (e.w & 511u) == b) {
            const uint32_t bs = base[b], k0 = 4u * v - ls[b];
            const uint32_t d = bs + k0;
            // the quad lies inside its bucket's run, and the run inside the batch
            if (k0 + 3u < cnt[b] && d + 4u <= P.n && d + 4u > d) {
                const u32x4 x = {p0 + (e.x >> 9), p0 + (e.y >> 9), p0 + (e.z >> 9),
                                 p0 + (e.w >> 9)};
                // non-temporal, whole lines and the partial lines at a run's
                // ends alike: plain stores for the partial lines left them
                // dirty in L2, written back inside the next batch's parse
                // kernel (+14 us there at 9 buckets, same box,
                // profiles/r03_ab_store.log); write-through (sc1) stores cost
                // the scatter 1.7-3.8x
                __builtin_nontemporal_store(x, reinterpret_cast<u32x4 *>(P.qidx + d));
                wrote += 4u;
            } else {
                report_fault(P.fault, YRSS_FAULT_LIST_RANGE, YRSS_K_SCATTER, p0 + (e.x >> 9), d);
            }
        } else {
            // a quad across a run boundary or padding: word by word
            auto one = [&](uint32_t w, uint32_t k) {
                const uint32_t bk = w & 511u;
                if (bk >= P.nb)
                    return;
                const uint32_t kk = 4u * v + k - ls[bk];
                const uint32_t d = base[bk] + kk;
                if (kk < cnt[bk] && d < P.n) {
                    P.qidx[d] = p0 + (w >> 9);
                    ++wrote;
                } else {
                    report_fault(P.fault, YRSS_FAULT_LIST_RANGE, YRSS_K_SCATTER, p0 + (w >> 9),
                                 d);
                }
            };
            one(e.x, 0u);
            one(e.y, 1u);
            one(e.z, 2u);
            one(e.w, 3u);
        }
    }
    return wrote;
}

__global__ __launch_bounds__(kScatterBlock, 4) void yrss_scatter(ScatterParams P)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint32_t lane = lane_id();
    const uint32_t wpb = blockDim.x / kWave;
    // per wave: start[nb] the lists' starts; base[nb] the piece's first list
    // slot per bucket; ls[nb] the bucket's run start in the stage; cnt[nb]
    // the piece's count per bucket; cur[nb] the placement cursors; send[nb]
    // the span's end per bucket; then the stage
    uint32_t *start = reinterpret_cast<uint32_t *>(smem) + wave * P.wlds;
    uint32_t *base = start + P.nb, *ls = base + P.nb, *cnt = ls + P.nb;
    uint32_t *cur = cnt + P.nb, *send = cur + P.nb;
    uint32_t *stg = start + P.aux;
    const uint32_t W = gridDim.x * wpb;
    const uint32_t gw = xcd_block(P.xcd) * wpb + wave;
    const uint32_t ng = (uint32_t)(((uint64_t)P.n + P.seg - 1u) / P.seg);
    // the lists' 16-byte phase: qidx + d is 16-byte aligned iff (d + ph) % 4 == 0
    const uint32_t ph = (uint32_t)(((uintptr_t)P.qidx >> 2) & 3u);

    // list starts (exclusive scan of totals); wave 0 also writes qstart
    uint32_t carry = 0, nzb = 0;
    for (uint32_t b0 = 0; b0 < P.nb; b0 += kWave) {
        const uint32_t b = b0 + lane;
        const uint32_t t = b < P.nb ? P.totals[b] : 0u;
        nzb += (uint32_t)__popcll(__ballot(t != 0u));
        const uint32_t x = wave_incl_scan(t, lane);
        if (b < P.nb) {
            start[b] = carry + x - t;
            cnt[b] = 0u;
            if (gw == 0)
                P.qstart[b] = carry + x - t;
        }
        carry += __shfl(x, kWave - 1, kWave);
    }
    if (gw == 0 && lane == 0)
        P.qstart[P.nb] = carry;
    const ListOut lout = list_out(P.qidx, P.n);
    if (nzb == 1) {
        // one non-empty list (all-UDP traffic): 0, 1, ..., n-1, grid-stride
        const uint32_t head = min(P.n, (4u - ph) & 3u);
        const uint32_t nv = (P.n - head) >> 2;
        const uint32_t T = gridDim.x * blockDim.x;
        const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
        if (id < head)
            list_store1<kListAux>(lout, id, id);
        for (uint32_t v = id; v < nv; v += T) {
            const uint32_t x = head + 4u * v;
            list_store4<kListAux>(lout, x, u32x4{x, x + 1u, x + 2u, x + 3u});
        }
        const uint32_t t = head + 4u * nv + id;
        if (t < P.n)
            list_store1<kListAux>(lout, t, t);
        return;
    }
    if (gw >= ng)
        return;
    auto prefix = [&](uint32_t b, uint32_t c) {
        return c < P.nchunk ? P.seg_off[(size_t)b * P.ncol + c] : P.totals[b];
    };
    auto span_end = [&](uint32_t g) {
        const uint64_t e = (uint64_t)g * P.seg + P.seg;
        return e < P.n ? (uint32_t)e : P.n;
    };
    // stage layout from cnt[]: bucket b's run at ls[b] == base[b] + ph (mod 4),
    // the rest padding (0xFFFFFFFF: bucket field 511 >= nb)
    auto layout = [&]() {
        uint32_t raw = 0;
        for (uint32_t b0 = 0; b0 < P.nb; b0 += kWave) {
            const uint32_t b = b0 + lane;
            const uint32_t w = b < P.nb ? cnt[b] + 3u : 0u;
            const uint32_t x = wave_incl_scan(w, lane);
            if (b < P.nb) {
                const uint32_t r = raw + x - w;
                ls[b] = r + ((base[b] + ph - r) & 3u);
            }
            raw += __shfl(x, kWave - 1, kWave);
        }
        for (uint32_t v = lane; v < P.stg / 4u; v += kWave)
            reinterpret_cast<u32x4 *>(stg)[v] = u32x4{~0u, ~0u, ~0u, ~0u};
    };
    wave_lds_sync();

    {
        uint32_t g = gw, p0 = gw * P.seg;
        uint32_t pe = min(span_end(g), p0 + kPiece);
        uint32_t qv[kPieceSlots], qn[kPieceSlots];
        load_piece(reinterpret_cast<const uint16_t *>(P.q), p0, pe, opaque(lane), qv);
        for (;;) {
            const uint32_t se = span_end(g);
            if (p0 == g * P.seg) {
                // a new span: its lists' first slots and, for the check at its
                // end, where each bucket's run must finish
                const uint32_t c0 = g << P.gshift, c1 = c0 + (1u << P.gshift);
                for (uint32_t b = lane; b < P.nb; b += kWave) {
                    base[b] = start[b] + prefix(b, c0);
                    send[b] = start[b] + prefix(b, c1);
                }
                wave_lds_sync();
            }
            // count
            rank_piece<false>(P, qv, p0, pe, lane, cnt, stg);
            wave_lds_sync();
            layout();
            for (uint32_t b = lane; b < P.nb; b += kWave)
                cur[b] = ls[b];
            wave_lds_sync();
            // place
            rank_piece<true>(P, qv, p0, pe, lane, cur, stg);
            // the next piece's q is in flight during the copy-out
            uint32_t g2 = g, p2 = pe;
            if (pe >= se) {
                g2 = g + W;
                p2 = g2 * P.seg;
            }
            const bool more = g2 < ng;
            const uint32_t pe2 = more ? min(span_end(g2), p2 + kPiece) : 0u;
            if (more)
                load_piece(reinterpret_cast<const uint16_t *>(P.q), p2, pe2, opaque(lane), qn);
            wave_lds_sync();
            (void)copy_out(P, stg, base, ls, cnt, p0, ph, lane);
            wave_lds_sync();
            // the next piece's lists start where this one's end
            for (uint32_t b = lane; b < P.nb; b += kWave) {
                base[b] += cnt[b];
                cnt[b] = 0u;
                if (pe >= se && base[b] != send[b])
                    report_fault(P.fault, YRSS_FAULT_COUNT_MISMATCH, YRSS_K_SCATTER, g, b);
            }
            wave_lds_sync();
            if (!more)
                break;
            g = g2;
            p0 = p2;
            pe = pe2;
#pragma unroll
            for (uint32_t k = 0; k < kPieceSlots; ++k)
                qv[k] = qn[k];
        }
    }
}

// ---------------------------------------------------------------------------
// Kernel 3 (ranked): the lists written in whole 64-byte lines.
//
// A workgroup takes one contiguous range of spans (a span: 2^gshift parse
// chunks, up to line_span_max(kG) packets) and works them in order.  Per span it
// places every packet in an LDS stage by the parse kernel's rank (stage slot =
// the bucket's position for its chunk + rank, the positions from the scan's
// prefixes), the stage laid out line for line like the lists: bucket b's
// words sit in stage lines of their own at their list address's phase inside
// a 64-byte line.  Whole lines go out as 16-byte non-temporal stores, four
// lanes to a line; the bucket's last line, when the span ends inside it, is
// carried in LDS into the next span's stage and completed there, so inside a
// workgroup's range every line leaves complete, once.  Only the first and last
// line of each bucket in a range can be partial (word stores).  A list line
// written in pieces costs a read-modify-write or a second partial write-back;
// the per-wave scatter this replaces wrote ~30-word runs per span at 64
// buckets and most of its lines in two pieces (r03 q-rows: 63 us scatter and
// +14 us in the next parse kernel, against the list-write floor of ~15 us).
//
// The packets' (bucket, rank) come from the parse kernel's rank stream: packed
// as bucket << cshift | rank when the bucket fits beside the rank (kPacked;
// the scatter then reads 2 bytes a packet), else the rank beside q.  Checks: a
// slot outside the stage lands in a spare word, a list position outside the
// batch is not stored, and the words a workgroup writes must add up to its
// range's packets with the sum of its range's packet indices (two packets on
// one slot leave another slot holding an earlier span's index); each reports
// through the fault record instead of storing (YRSS_FAULT_STAGE /
// _LIST_RANGE / _COUNT_MISMATCH).
// ---------------------------------------------------------------------------
constexpr int kLineBlock = 512;
// s_waitcnt vmcnt(0), expcnt and lgkmcnt left alone (gfx9 encoding)
constexpr int kWaitVm0 = 0x0F70;
// prefix words a thread holds: the table is nb x span chunks <= 512 x regs
// words (2048 at default chunks: 128 buckets x 16 chunks; more only when
// chunk_tiles is forced small, where the span gets fewer chunks instead)
constexpr uint32_t line_tab_regs(uint32_t g) { return g == 2u ? 5u : 9u; }
constexpr uint32_t line_tab_max(uint32_t g) { return kLineBlock * line_tab_regs(g); }
// A span is kG 8-packet groups a thread: 8192 packets (kG = 2) up to 128
// buckets, 16384 (kG = 4) past that, where the per-bucket work of a span
// (carried lines, layout) is large enough to amortise over twice the packets
// (q255 scatter 93 -> 75 us; at 64 buckets kG = 4 cost 3-4 us, r03 A/B).
constexpr uint32_t line_span_max(uint32_t g) { return kLineBlock * 8u * g; }
// Wave 0 holds the per-bucket totals and span prefixes a bucket to a lane, in
// line_bucket_regs(kG) registers each: the kernel serves nb <= 64 x that.
// A launch past it would leave the other buckets' layout words unwritten, and
// the tagging loop bounded by them would run ~2^31 iterations of dropped LDS
// stores (round 4's hang): the host refuses such a plan
// (-EINVAL) and the kernel checks again at entry.
constexpr uint32_t line_bucket_regs(uint32_t g) { return g == 2u ? 2u : 8u; }
constexpr uint32_t line_nb_max(uint32_t g) { return 64u * line_bucket_regs(g); }
// In-scatter prefixes (LineParams.fused) up to 16 buckets: the scan kernel and
// its launch gap leave the step.  Waves 1-7 of a workgroup take a bucket row
// each (up to kFusedRows): its counts over the range's chunks and its bins of
// the earlier ranges; the range bins are [nb][kLbMaxWgs].
constexpr uint32_t kFusedMaxNb = 16;
// the bucket-major tagging is kept while no thread gets more than kTagIters
// of a bucket's lines
constexpr uint32_t kTagIters = 6;
constexpr uint32_t kFusedRows = 3;          // bucket rows a loading wave (waves 1-7)
constexpr uint32_t kFusedMaxCols = 256;      // chunks a range: 4 a lane
constexpr uint32_t kFusedMaxRanges = 512;    // earlier ranges' bins: 8 a lane
static_assert(line_nb_max(4) <= (uint32_t)kLineBlock, "tagging: a thread to a bucket at least");


struct LineParams {
    const int16_t *q;          // !kPacked: the bucket of each packet
    const uint16_t *rank;      // rank in chunk (kPacked: bucket << cshift | rank)
    const uint32_t *seg_off;   // [nb][ncol] exclusive per-bucket prefix per chunk
    const uint32_t *totals;    // [nb]
    uint32_t *qidx;
    uint32_t *qstart;          // [nb + 1]
    uint32_t *fault;
    uint32_t n, nq, nb, nchunk, ncol;
    uint32_t seg;              // packets per span: 2^gshift chunks, <= line_span_max(kG)
    uint32_t gshift, cshift;   // span = 2^gshift chunks, chunk = 2^cshift packets
    uint32_t lmax;             // stage lines: seg / 16 + 2 nb + 1
    uint32_t xcd;              // workgroups of one XCD take consecutive ranges
    uint32_t nt;               // list stores non-temporal only (no sc1): past 64 buckets
                               // (the instantiation's kNt; the host picks it from this)
    uint32_t early;            // first span's loads before the totals: past 16 buckets
    uint32_t merge;            // partial lines (a range's first / last) as plain stores: L2 merges
    // In-scatter prefixes (fused, up to kFusedMaxNb buckets): no scan kernel
    // runs.  The parse kernel sums the totals and, per scatter range of rcs
    // spans, the range's counts (range bins); each workgroup scans its own
    // range's chunk counts in LDS from the sum of the earlier ranges' bins.
    const uint32_t *cnt;       // [nb][ncol] per-chunk counts (the parse kernel's)
    const uint32_t *rbin;      // [nb][kLbMaxWgs] range bins (the parse kernel's)
    uint32_t *tot_next;        // the next batch's totals set: zeroed here
    uint32_t *rbin_next;       // the next batch's range bins: zeroed here
    uint32_t fused;
    uint32_t rcs;              // spans a range
    uint32_t rts;              // row stride of the range table: range chunks + 1
};

// LDS of a workgroup, in words: per-bucket arrays, the prefix table, the
// carried lines, the stage's line tags, the stage (+ a spare word); with
// in-scatter prefixes also the range table.
struct LineLds {
    uint32_t start, cs, ve, ce, so, rb, lsl, misc, tab, cb, ltag, lgl, stg, rt, words;
};
__host__ __device__ inline LineLds line_lds(uint32_t nb, uint32_t gshift, uint32_t lmax,
                                            uint32_t rts = 0)
{
    LineLds L;
    uint32_t o = 0;
    auto take = [&](uint32_t w) {
        const uint32_t at = o;
        o = (o + w + 3u) & ~3u;
        return at;
    };
    // the per-bucket layout arrays come in two sets, a span's and the next's
    L.start = take(nb);
    L.cs = take(2u * nb);    // the span's first valid list position (adjusted), carry start
    L.ve = take(2u * nb);    // the span's end position (adjusted)
    L.ce = take(2u * nb);    // carry end = the span's first packet position (adjusted)
    L.so = take(2u * nb);    // stage index = so[b] + adjusted position
    L.rb = take(2u * nb);    // prefix table row bias (to stage slots)
    L.lsl = take(2u * (nb + 1u));   // first stage line of each bucket
    L.misc = take(10);   // [8 + s]: the tagging's form for layout set s
    L.tab = take(nb * ((1u << gshift) + 1u));   // rows of 2^gshift + 1 words (odd: banks)
    L.cb = take(16u * nb);
    L.ltag = take(lmax);  // bucket | copy mode << 30 per stage line
    L.lgl = take(lmax);   // the line's list line (adjusted position / 16)
    L.stg = take(16u * lmax + 4u);
    L.rt = take(nb * rts);   // [nb][rts]: the range's chunk prefixes, then its end
    L.words = o;
    return L;
}

// 8 x 16-bit words per 16-byte load, groups k = 0, 1 of this thread: packets
// p0 + 8 (512 k + t) ..+7; past pe read 0 (range check; a batch's last span
// that ends inside a vector is read word by word, as the check drops a
// partial vector whole).
template <uint32_t kG>
__device__ __forceinline__ void load_groups(const uint16_t *a, uint32_t p0, uint32_t pe,
                                            uint32_t t, u32x4 (&v)[kG])
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(a + p0), 0, (int)((pe - p0) * 2u), kRsrcWord3);
    if (((pe - p0) & 7u) == 0) {
#pragma unroll
        for (uint32_t k = 0; k < kG; ++k)
            v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 r, (int)((k * kLineBlock + t) * 16u), 0, 2));
    } else {
#pragma unroll
        for (uint32_t k = 0; k < kG; ++k) {
            uint32_t w[4];
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) {
                const int o = (int)((k * kLineBlock + t) * 16u + 4u * i);
                w[i] = __builtin_amdgcn_raw_buffer_load_b16(r, o, 0, 0) |
                       ((uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, o + 2, 0, 0) << 16);
            }
            v[k] = u32x4{w[0], w[1], w[2], w[3]};
        }
    }
}

// the line scatter's phase clock (LPROF, LPROF_ENTRY): no-ops outside
// measurement builds (tools/build_ab_lib.sh prof)
#include "yrss_line_prof.h"

template <bool kPacked, uint32_t kG, bool kNt>
__global__ __launch_bounds__(kLineBlock, kG == 4u ? 2 : 4) void yrss_scatter_lines(LineParams P)
{
    // list stores: non-temporal only past kListNtBuckets buckets, else nt | sc1
    constexpr int kNtAux = kNt ? kListAuxMany : kListAux;
    extern __shared__ __attribute__((aligned(16))) uint32_t lsm[];
    const uint32_t nb = P.nb, t = threadIdx.x, lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(t / kWave);
    // Capacity, checked before any barrier (the condition is uniform): a
    // plan past what this instantiation holds reports and leaves, instead of
    // running on unwritten per-bucket words (see line_nb_max)
    if (nb > line_nb_max(kG) || (nb << P.gshift) > line_tab_max(kG) ||
        P.lmax > kLineBlock * (kG == 4u ? 5u : 2u)) {
        if (t == 0)
            report_fault(P.fault, YRSS_FAULT_LINE_CAPACITY, YRSS_K_SCATTER, nb, line_nb_max(kG));
        return;
    }
    const LineLds o = line_lds(nb, P.gshift, P.lmax, P.fused ? P.rts : 0u);
    LPROF_ENTRY();
    uint32_t *start = lsm + o.start, *cs = lsm + o.cs, *ve = lsm + o.ve, *ce = lsm + o.ce;
    uint32_t *so = lsm + o.so, *rb = lsm + o.rb, *lsl = lsm + o.lsl;
    uint32_t *misc = lsm + o.misc, *tab = lsm + o.tab, *cb = lsm + o.cb, *ltag = lsm + o.ltag;
    uint32_t *lgl = lsm + o.lgl;
    uint32_t *stg = lsm + o.stg;
    uint32_t *const cs_sets = cs, *const ve_sets = ve, *const ce_sets = ce, *const so_sets = so;
    uint32_t *const lsl_sets = lsl;
    const uint32_t cap = 16u * P.lmax;   // the spare word
    // list position x is "adjusted" a = x + ph: 64-byte lines are a >> 4
    const uint32_t ph = (uint32_t)(((uintptr_t)P.qidx >> 2) & 15u);

    // this workgroup's range of spans
    const uint32_t nsp = (uint32_t)(((uint64_t)P.n + P.seg - 1u) / P.seg);
    // (in-scatter prefixes: ranges of rcs spans in blockIdx order, the
    // partition the parse kernel's range bins were summed by)
    const uint32_t r = P.fused ? blockIdx.x : xcd_block(P.xcd), G = gridDim.x;
    const uint32_t g0 = P.fused ? min(r * P.rcs, nsp) : (uint32_t)((uint64_t)r * nsp / G);
    const uint32_t g1 = P.fused ? min(g0 + P.rcs, nsp) : (uint32_t)((uint64_t)(r + 1u) * nsp / G);
    if (P.fused) {
        // the next batch's totals and range bins start from zero (no one
        // reads them in this kernel; each workgroup clears a slice)
        if (blockIdx.x == 0 && t < nb)
            P.tot_next[t] = 0u;
        const uint32_t zw = kLbMaxWgs * nb, per = (zw + G - 1u) / G;
        for (uint32_t e = r * per + t; e < min(zw, (r + 1u) * per); e += kLineBlock)
            P.rbin_next[e] = 0u;
    }
    // prefix table rows are ncs + 1 words apart: with a power-of-two row the
    // lanes of one chunk column hit one or two LDS banks whatever their bucket
    // (a 0.78 conflict share of the LDS cycles at 64 buckets)
    const uint32_t ncs = 1u << P.gshift, ntab = nb << P.gshift, rs = ncs + 1u;
    auto prefix = [&](uint32_t b, uint32_t c) {
        return c < P.nchunk ? P.seg_off[(size_t)b * P.ncol + c] : P.totals[b];
    };
    auto span_end = [&](uint32_t g) {
        const uint64_t e = (uint64_t)g * P.seg + P.seg;
        return e < P.n ? (uint32_t)e : P.n;
    };
    // set 1 holds the state before the range's first span (set 0): its
    // prefixes are loaded beside the first span's streams (one round trip for
    // both) and written once they have arrived
    uint32_t pre0 = 0;
    const __amdgpu_buffer_rsrc_t lout = line_out(P.qidx, P.n);
    // The span's streams alternate between two register sets: span g+1's
    // loads issue at the start of span g's phase (b), once its table is in
    // LDS, and are waited for just before span g's copy-out.  vmcnt counts
    // loads and stores in one in-order queue, so a load issued before a
    // span's list stores and waited for after them waits for those stores
    // too (their write-through acks), and a load issued after the place phase
    // had only the copy-out to hide its latency.
    u32x4 pkA[kG], qkA[kG], pkB[kG], qkB[kG];
    // wave 0 also holds, a bucket to a lane, each bucket's prefix at the
    // span's first chunk and at its end, so it lays the span out from
    // registers while the other waves write the prefix table
    constexpr uint32_t kBI = line_bucket_regs(kG);   // nb <= 64 kBI (checked at entry)
    constexpr uint32_t kLineTabRegs = line_tab_regs(kG);
    uint32_t pt[kLineTabRegs], w0s[kBI], w0e[kBI];
    uint32_t crn = 0;   // in-scatter prefixes: the range's chunks (range table columns)
    // (fused: `part` 1 the LDS prefixes only, 2 the streams only, 3 both)
    auto load_span = [&](uint32_t g, u32x4 (&pk)[kG], u32x4 (&qk)[kG], uint32_t part = 3u) {
        const uint32_t p0 = g * P.seg, pe = span_end(g), tt = opaque(t);
        const uint32_t c0 = g << P.gshift;
        if (P.fused && (part & 1u)) {
            // the prefixes from the range table in LDS (written once, in the
            // prologue); the range's last span ends at the range's end column
            const uint32_t *rt = lsm + o.rt;
            const uint32_t j0 = c0 - (g0 << P.gshift), je = min(j0 + ncs, crn);
            if (wave == 0) {
                const uint32_t ll = opaque(lane);
#pragma unroll
                for (uint32_t i = 0; i < kBI; ++i) {
                    if (i * kWave < nb) {   // (uniform)
                        const uint32_t b = min(i * kWave + ll, nb - 1u);
                        w0s[i] = rt[b * P.rts + j0];
                        w0e[i] = rt[b * P.rts + je];
                    }
                }
            }
#pragma unroll
            for (uint32_t k = 0; k < kLineTabRegs; ++k) {
                const uint32_t e = min(k * kLineBlock + tt, ntab - 1u);
                if (k * kLineBlock < ntab)   // (uniform)
                    pt[k] = rt[(e >> P.gshift) * P.rts + j0 + (e & (ncs - 1u))];
            }
        }
        if (P.fused) {
            if (part & 2u) {
                load_groups(P.rank, p0, pe, tt, pk);
                if (!kPacked)
                    load_groups(reinterpret_cast<const uint16_t *>(P.q), p0, pe, tt, qk);
            }
            return;
        }
        // the prefixes first, the streams last: vmcnt counts in issue order,
        // so the prologue can wait for the prefixes alone (the first span's
        // layout and table then overlap its streams' arrival)
        if (part & 1u) {
        if (wave == 0) {
            // rows past nb read 0 (range check); a span's end past the last
            // chunk is the bucket's total
            const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint32_t *>(P.seg_off), 0, (int)(nb * P.ncol * 4u), kRsrcWord3);
            const __amdgpu_buffer_rsrc_t rtot = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint32_t *>(P.totals), 0, (int)(nb * 4u), kRsrcWord3);
            const bool inner = c0 + ncs < P.nchunk;
            const uint32_t ll = opaque(lane);
#pragma unroll
            for (uint32_t i = 0; i < kBI; ++i) {
                if (i * kWave < nb) {   // (uniform)
                    const uint32_t b = i * kWave + ll;
                    w0s[i] = __builtin_amdgcn_raw_buffer_load_b32(rs0, (int)(b * P.ncol * 4u),
                                                                  (int)(c0 * 4u), 0);
                    w0e[i] = inner ? __builtin_amdgcn_raw_buffer_load_b32(
                                         rs0, (int)(b * P.ncol * 4u), (int)((c0 + ncs) * 4u), 0)
                                   : __builtin_amdgcn_raw_buffer_load_b32(rtot, (int)(b * 4u), 0, 0);
                }
            }
        }
        // element k * 512 + t is row (t >> gshift) + k * (512 >> gshift),
        // column t & (ncs - 1), so one per-lane offset and a scalar step per
        // k; rows past nb read 0 (range check).  Columns past the last chunk
        // (a batch's last span) read whatever the matrix holds there: no
        // packet's slot uses them.  One load form on every path: a plain
        // load on a rare path left a pending destination register that the
        // compiler later waited for with vmcnt(0), i.e. for every list store
        // in flight.
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t *>(P.seg_off), 0, (int)(nb * P.ncol * 4u), kRsrcWord3);
        const uint32_t vo = ((tt >> P.gshift) * P.ncol + (tt & (ncs - 1u))) * 4u;
        const uint32_t step = (kLineBlock >> P.gshift) * P.ncol * 4u;
#pragma unroll
        for (uint32_t k = 0; k < kLineTabRegs; ++k)
            if (k * kLineBlock < ntab)   // (uniform)
                pt[k] = __builtin_amdgcn_raw_buffer_load_b32(r, (int)vo,
                                                             (int)(c0 * 4u + k * step), 0);
        }
        if (part & 2u) {
            load_groups(P.rank, p0, pe, tt, pk);
            if (!kPacked)
                load_groups(reinterpret_cast<const uint16_t *>(P.q), p0, pe, tt, qk);
        }
    };
    // list starts (exclusive scan of totals); workgroup 0 also writes qstart.
    // Every bucket block's total is loaded before the first is scanned: one
    // round trip, not one per 64 buckets.  The totals go first: waiting for
    // them must not wait for the first span's streams behind them.
    constexpr uint32_t kTB = line_bucket_regs(kG);   // nb <= 64 kTB (checked at entry)
    uint32_t tv[kTB];
    auto load_totals = [&]() {   // (wave 0)
        const __amdgpu_buffer_rsrc_t rt_ = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t *>(P.totals), 0, (int)(nb * 4u), kRsrcWord3);
#pragma unroll
        for (uint32_t i = 0; i < kTB; ++i)
            tv[i] = i * kWave < nb ? __builtin_amdgcn_raw_buffer_load_b32(
                                         rt_, (int)((i * kWave + lane) * 4u), 0, 0)
                                   : 0u;
    };
    auto scan_totals = [&]() {   // (wave 0)
        uint32_t carry = 0, nzb = 0;
#pragma unroll
        for (uint32_t i = 0; i < kTB; ++i) {
            if (i * kWave >= nb)   // (uniform)
                break;
            const uint32_t b = i * kWave + lane;
            const uint32_t x0 = tv[i];
            nzb += (uint32_t)__popcll(__ballot(x0 != 0u));
            const uint32_t x = wave_incl_scan(x0, lane);
            if (b < nb) {
                start[b] = carry + x - x0;
                if (blockIdx.x == 0)
                    P.qstart[b] = carry + x - x0;
            }
            carry += __shfl(x, kWave - 1, kWave);
        }
        if (lane == 0) {
            if (blockIdx.x == 0)
                P.qstart[nb] = carry;
            misc[0] = nzb;
            misc[1] = 0u;
            misc[3] = 0u;
        }
        LPROF_PRO(1);
    };
    // In-scatter prefixes: waves 1-7 take the bucket rows b = wave - 1,
    // wave + 6, ... (nb <= 16: three at most) and load, a lane 16 bytes at a
    // time, the row's counts over the range's chunks (crn <= 256 columns) and
    // its bins of every earlier range (r <= 512), while wave 0 loads and
    // scans the totals.  Nine 16-byte loads a lane at most, no divisions:
    // the waves reach the one-list barrier at once, and wave 0 waits for the
    // totals alone (its loads and their use sit in one branch: split in two,
    // the compiler waited for every load of the other waves' path at the
    // barrier), so the one-list path is not held up by these loads.
    constexpr uint32_t kFR = kFusedRows;
    u32x4 fc[kFR], fb0[kFR], fb1[kFR];
    if (P.fused) {
        const uint32_t cr0 = g0 << P.gshift;
        crn = g0 < g1 ? min(g1 << P.gshift, P.nchunk) - cr0 : 0u;
    }
    if (P.early) {
        // Past 16 buckets the first span's prefixes and streams are issued
        // after the totals and before they are scanned, so the round trips
        // overlap (such batches are rarely one-list, where these loads go
        // unused)
        if (wave == 0)
            load_totals();
        if (g0 < g1) {
            pre0 = t < nb ? prefix(t, g0 << P.gshift) : 0u;
            load_span(g0, pkA, qkA);
        }
        if (wave == 0)
            scan_totals();
    } else if (wave == 0) {
        load_totals();
        scan_totals();
    } else if (P.fused) {
        const uint32_t cr0 = g0 << P.gshift;
        const __amdgpu_buffer_rsrc_t rc_ = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t *>(P.cnt), 0, (int)(nb * P.ncol * 4u), kRsrcWord3);
        const __amdgpu_buffer_rsrc_t rb_ = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t *>(P.rbin), 0, (int)(nb * kLbMaxWgs * 4u), kRsrcWord3);
#pragma unroll
        for (uint32_t k = 0; k < kFR; ++k) {
            const uint32_t b = wave - 1u + k * (kLineBlock / kWave - 1u);
            const uint32_t bo = b < nb ? b : nb;   // rows past nb: past the range, read 0
            // (lanes past the range's columns or the earlier ranges read past
            // the buffer: the range check returns 0 and nothing is fetched,
            // which a one-list batch, where these go unused, would pay for)
            constexpr uint32_t kOut = 0x7ffffff0u;
            fc[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                rc_, (int)(4u * lane < crn ? (bo * P.ncol + cr0 + 4u * lane) * 4u : kOut), 0, 0));
            fb0[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                rb_, (int)(8u * lane < r ? (bo * kLbMaxWgs + 8u * lane) * 4u : kOut), 0, 0));
            fb1[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                rb_, (int)(8u * lane + 4u < r ? (bo * kLbMaxWgs + 8u * lane + 4u) * 4u : kOut),
                0, 0));
        }
    }
    __syncthreads();
    LPROF_PRO(2);
    if (misc[0] == 1u) {
        // one non-empty list (all-UDP traffic): 0, 1, ..., n-1, grid-stride
        // 16-byte non-temporal stores (64 MB in 10.7 us,
        // profiles/r02_v8_hbm_write.log)
        const __amdgpu_buffer_rsrc_t lo = line_out(P.qidx, P.n);
        const uint32_t ph4 = ph & 3u;
        const uint32_t head = min(P.n, (4u - ph4) & 3u);
        const uint32_t nv = (P.n - head) >> 2;
        const uint32_t T = gridDim.x * blockDim.x;
        const uint32_t id = blockIdx.x * blockDim.x + t;
        if (id < head)
            line_store1<kListAux>(lo, id, id);
        for (uint32_t v = id; v < nv; v += T) {
            const uint32_t x = head + 4u * v;
            line_store4<kListAux>(lo, x, u32x4{x, x + 1u, x + 2u, x + 3u});
        }
        const uint32_t e = head + 4u * nv + id;
        if (e < P.n)
            line_store1<kListAux>(lo, e, e);
        return;
    }

    if (P.fused) {
        // In-scatter prefixes, from what the parse kernel left (all of it
        // complete when this kernel starts, so no workgroup waits on another):
        // the range's chunk counts go into the range table, the earlier
        // ranges' bins add up to the range's base per bucket, and a wave to a
        // bucket row scans the row starting from that base; column crn gets
        // the range's end.  Every span's prefixes then come from LDS.
        uint32_t *rt = lsm + o.rt;
        if (wave != 0) {
            // a row: the bins of the ranges before this one (words past r
            // masked) add up to the row's base; the counts (words past crn
            // masked), scanned across the wave from that base, are the row's
            // exclusive prefixes; column crn gets the range's end
#pragma unroll
            for (uint32_t k = 0; k < kFR; ++k) {
                const uint32_t b = wave - 1u + k * (kLineBlock / kWave - 1u);
                if (b >= nb)   // (uniform)
                    break;
                const uint32_t q0 = 8u * lane;
                const uint32_t bins = (q0 + 0u < r ? fb0[k].x : 0u) + (q0 + 1u < r ? fb0[k].y : 0u) +
                                      (q0 + 2u < r ? fb0[k].z : 0u) + (q0 + 3u < r ? fb0[k].w : 0u) +
                                      (q0 + 4u < r ? fb1[k].x : 0u) + (q0 + 5u < r ? fb1[k].y : 0u) +
                                      (q0 + 6u < r ? fb1[k].z : 0u) + (q0 + 7u < r ? fb1[k].w : 0u);
                const uint32_t base = __shfl(wave_incl_scan(bins, lane), kWave - 1, kWave);
                const uint32_t c0 = 4u * lane;
                const uint32_t x0 = c0 + 0u < crn ? fc[k].x : 0u, x1 = c0 + 1u < crn ? fc[k].y : 0u;
                const uint32_t x2 = c0 + 2u < crn ? fc[k].z : 0u, x3 = c0 + 3u < crn ? fc[k].w : 0u;
                const uint32_t sum = x0 + x1 + x2 + x3;
                const uint32_t inc = wave_incl_scan(sum, lane);
                const uint32_t tot = __shfl(inc, kWave - 1, kWave);   // (every lane: a shuffle)
                uint32_t *row = rt + b * P.rts;
                uint32_t run = base + inc - sum;
                if (c0 + 0u < crn) row[c0 + 0u] = run;
                run += x0;
                if (c0 + 1u < crn) row[c0 + 1u] = run;
                run += x1;
                if (c0 + 2u < crn) row[c0 + 2u] = run;
                run += x2;
                if (c0 + 3u < crn) row[c0 + 3u] = run;
                if (lane == 0)
                    row[crn] = base + tot;
            }
        }
        // the first span's streams, after the rows (whose loads are then
        // waited for alone), in flight under the first layout
        if (g0 < g1)
            load_span(g0, pkA, qkA, 2u);
        __syncthreads();
        LPROF_PRO(3);
    }
    if (g0 >= g1)
        return;
    if (P.fused) {
        pre0 = t < nb ? lsm[o.rt + t * P.rts] : 0u;
        load_span(g0, pkA, qkA, 1u);
    } else if (!P.early) {
        pre0 = t < nb ? prefix(t, g0 << P.gshift) : 0u;
        load_span(g0, pkA, qkA);
    }
    // the first span's prefixes waited for here, its streams (issued last,
    // kG 16-byte loads a stream, more on a ragged span) left in flight under
    // the first layout and table
    __builtin_amdgcn_s_waitcnt(kWaitVm0 | (int)(kPacked ? kG : 2u * kG));
    if (t < nb) {
        const uint32_t a = start[t] + pre0 + ph;
        cs[nb + t] = a;
        ve[nb + t] = a;
    }
    // Wave 0, a bucket to a lane, lays span g out into set s from set s ^ 1
    // and the prefixes it holds (w0s, w0e): the valid positions [cs, ve) =
    // the carried words and the span's packets, the bucket's stage lines
    // (exclusive scan), its stage offset so and the bias rb from a prefix to
    // a stage slot.  Span g + 1's layout is made at the end of span g's
    // placement, as soon as its prefixes arrive, so a span starts with its
    // layout and table in place.
    auto layout = [&](uint32_t g, uint32_t s) {
        const uint32_t *pcs = cs + (s ^ 1u) * nb, *pve = ve + (s ^ 1u) * nb;
        uint32_t *wcs = cs + s * nb, *wve = ve + s * nb, *wce = ce + s * nb, *wso = so + s * nb;
        uint32_t *wrb = rb + s * nb, *wlsl = lsl + s * (nb + 1u);
        uint32_t lines = 0, mx = 0;   // mx: a bucket's most stage lines
        bool cut = false;   // a bucket's first valid position not on a quad: cut quads
        // (lane hidden from the optimiser: the per-lane LDS addresses of
        // both sets were hoisted out of the span loop and spilled)
        const uint32_t ll = opaque(lane);
#pragma unroll
        for (uint32_t i = 0; i < kBI; ++i) {
            if (i * kWave >= nb)   // (uniform)
                break;
            const uint32_t b = i * kWave + ll;
            uint32_t nl = 0, v0 = 0, e0 = 0;
            if (b < nb) {
                e0 = pve[b];
                v0 = max(pcs[b], e0 & ~15u);
                const uint32_t e1 = e0 + (w0e[i] - w0s[i]);
                wcs[b] = v0;
                wce[b] = e0;
                wve[b] = e1;
                nl = ((e1 + 15u) >> 4) - (v0 >> 4);
            }
            const uint32_t x = wave_incl_scan(nl, lane);
            if (b < nb) {
                const uint32_t l0 = lines + x - nl;
                wlsl[b] = l0;
                wso[b] = 16u * (l0 - (v0 >> 4));
                wrb[b] = 16u * (l0 - (v0 >> 4)) + e0 - w0s[i];
            }
            lines += __shfl(x, kWave - 1, kWave);
            cut |= __ballot(b < nb && (v0 & 3u) != 0u) != 0ull;
            mx = max(mx, nl);
        }
        if (kG == 4u) {   // (the skewed form is built past 128 buckets only: in
                          // the kG = 2 kernel its code cost 0.6-1 us a batch at
                          // 4-9 buckets, profiles/r06_ab_c11_*, r06_ab_c12_*)
#pragma unroll
            for (uint32_t d = 1; d < (uint32_t)kWave; d <<= 1)
                mx = max(mx, (uint32_t)__shfl_xor(mx, d, kWave));
        } else {
            mx = 0u;
        }
        if (lane == 0) {
            if (lines > P.lmax) {
                report_fault(P.fault, YRSS_FAULT_STAGE, YRSS_K_SCATTER, g, lines);
                lines = 0;
            }
            wlsl[nb] = lines;
            misc[4u + s] = lines;
            misc[6u + s] = cut ? 1u : 0u;
            // a thread to a bucket's lines unless that leaves some thread more
            // than kTagIters of them (one bucket holding most of the traffic)
            misc[8u + s] = mx > kTagIters * (kLineBlock / nb) ? 1u : 0u;
        }
    };
    // span g's prefix table, tab[b][c] = prefix at chunk c + rb[b] (rows of
    // ncs + 1 words, every thread its prefix words pt): a packet's stage slot
    // is then tab[b][chunk] + rank
    auto write_tab = [&](uint32_t s) {
        const uint32_t *rbs = rb + s * nb;
        const uint32_t tt = opaque(t);   // (addresses not hoisted out of the span loop: spills)
#pragma unroll
        for (uint32_t k = 0; k < kLineTabRegs; ++k) {
            const uint32_t e = k * kLineBlock + tt;
            if (k * kLineBlock < ntab && e < ntab)
                tab[(e >> P.gshift) * rs + (e & (ncs - 1u))] = pt[k] + rbs[e >> P.gshift];
        }
    };
    __syncthreads();   // set 1 written
    if (wave == 0)
        layout(g0, 0u);
    __syncthreads();
    LPROF_PRO(4);
    write_tab(0u);
    // nothing pending at the loop head: a pending load there made the
    // compiler wait vmcnt(0) at a first use in every span, i.e. for the
    // previous span's list stores as well
    __builtin_amdgcn_s_waitcnt(kWaitVm0);
    LPROF_PRO(5);
    __syncthreads();
    // words written and their sum: a range is complete iff it wrote each of
    // its packets once, so the sum must be that of its packet indices (two
    // packets on one slot leave another slot with an earlier span's index)
    uint32_t wrote = 0, wsum = 0;
    // the tagging: a thread to a bucket's lines (bucket tb, lines tj + k tk),
    // or, on skewed spans, a thread to lines t + 512 k with the binary
    // search's first step tag_hi (the highest power of two below nb);
    // lmax <= 512 kTagLines
    const uint32_t tk = kLineBlock / nb, tb = t % nb, tj = t / nb;
    const uint32_t tag_hi = nb > 1u ? 1u << (31u - __builtin_clz(nb - 1u)) : 0u;
    constexpr uint32_t kTagLines = kG == 4u ? 5u : 2u;
    // the small per-bucket loops (carried words, cut quads, carry) start at
    // the last thread: wave 0 already lays the next span out and holds the
    // span's critical path
    const uint32_t tr = kLineBlock - 1u - t;
    auto span = [&](uint32_t g, uint32_t s, const u32x4 (&pk)[kG], const u32x4 (&qk)[kG],
                    u32x4 (&pkn)[kG], u32x4 (&qkn)[kG]) {
        const uint32_t p0 = g * P.seg, len = span_end(g) - p0;
        const bool last = g + 1u == g1;
        const uint32_t *cs = cs_sets + s * nb, *ve = ve_sets + s * nb, *ce = ce_sets + s * nb;
        const uint32_t *so = so_sets + s * nb;
        const uint32_t *lsl = lsl_sets + s * (nb + 1u);
        LPROF(0);
        // (the table was written in the previous span's copy-out, or the
        // prologue: two barriers a span)
        const uint32_t L = __builtin_amdgcn_readfirstlane(misc[4u + s]);
        // (b) three independent writes into LDS, no barrier between them:
        // - each stage line tagged with its bucket, list line and copy mode
        //   (0 whole, 1 carried, 2 word by word): thread t tags lines tj,
        //   tj + tk, ... of bucket tb (tk = 512 / nb threads to a bucket), one
        //   read of the bucket's bounds, then stores (a per-line binary search
        //   over the buckets' first lines was a chain of log2 nb dependent LDS
        //   reads; a wave per bucket walked nb / 8 buckets in turn);
        // - the carried words into their stage slots;
        // - every packet at slot = tab[b][chunk] + rank.
        if (!last)
            load_span(g + 1u, pkn, qkn);
        if (kG != 4u || !misc[8u + s]) {
            // a thread to a bucket's lines: lines tj, tj + tk, ... of bucket tb
            // (tk = 512 / nb threads to a bucket), one read of the bucket's
            // bounds, then stores
            const uint32_t b = opaque(tb);   // (addresses not hoisted: registers)
            if (tj < tk) {
                // (bounded by the span's line count whatever the words say)
                const uint32_t l0 = lsl[b], l1 = L ? min(lsl[b + 1u], L) : 0u, v0 = cs[b],
                               e1 = ve[b];
                for (uint32_t l = l0 + tj; l < l1; l += tk) {
                    const uint32_t gl = l - l0 + (v0 >> 4);
                    const uint32_t mode = 16u * gl >= v0 && 16u * gl + 16u <= e1 ? 0u
                                          : !last && gl == (e1 >> 4) && (e1 & 15u) != 0u ? 1u
                                                                                          : 2u;
                    ltag[l] = b | mode << 30;
                    lgl[l] = gl;
                }
            }
        } else {
            // skewed buckets (layout's misc[8 + s]): a thread to each of stage
            // lines t, t + 512, ... (< L), its
            // bucket found by a binary search over the buckets' first lines,
            // the searches of a thread's lines interleaved (their LDS reads
            // independent): balanced whatever the buckets' sizes.  A thread
            // to a bucket's lines (512 / nb threads a bucket) left one bucket
            // holding most of the traffic to a few threads: IMIX at 256
            // buckets, every UDP packet in queue 2, spent 22.7 us a span
            // tagging against 3.2 for all-TCP (profiles/r06_lineprof_skew_*);
            // on balanced buckets the search's log2 nb LDS round trips cost
            // more than the bucket-major loop (all-TCP at 256 buckets: scatter
            // 50 -> 58 us, profiles/r06_ab_c10_*), hence the choice a span
            uint32_t lb[kTagLines];
#pragma unroll
            for (uint32_t i = 0; i < kTagLines; ++i)
                lb[i] = 0u;
            for (uint32_t st = tag_hi; st; st >>= 1) {
#pragma unroll
                for (uint32_t i = 0; i < kTagLines; ++i) {
                    const uint32_t l = t + i * kLineBlock, c = lb[i] + st;
                    if (c < nb && lsl[c] <= l)
                        lb[i] = c;
                }
            }
#pragma unroll
            for (uint32_t i = 0; i < kTagLines; ++i) {
                const uint32_t l = t + i * kLineBlock;
                // (bounded by the span's line count whatever the words say)
                if (l < L) {
                    const uint32_t b = lb[i];
                    const uint32_t l0 = lsl[b], v0 = cs[b], e1 = ve[b];
                    const uint32_t gl = l - l0 + (v0 >> 4);
                    const uint32_t mode = 16u * gl >= v0 && 16u * gl + 16u <= e1 ? 0u
                                          : !last && gl == (e1 >> 4) && (e1 & 15u) != 0u ? 1u
                                                                                          : 2u;
                    ltag[l] = b | mode << 30;
                    lgl[l] = gl;
                }
            }
        }
        // the carried words, a quad a thread (a 16-byte copy where the quad
        // is whole and its stage slots aligned, else word by word: a whole-quad
        // write past ce would race the placement of the span's own packets)
        for (uint32_t e = tr; e < 4u * nb; e += kLineBlock) {
            const uint32_t b = e >> 2, q4 = 4u * (e & 3u);
            const uint32_t n = ce[b] - cs[b], base = so[b] + cs[b];
            if (q4 >= n)
                continue;
            if (q4 + 4u <= n && ((base + q4) & 3u) == 0u && base + q4 + 4u <= cap) {
                reinterpret_cast<u32x4 *>(stg)[(base + q4) >> 2] =
                    reinterpret_cast<const u32x4 *>(cb)[4u * b + (q4 >> 2)];
            } else {
#pragma unroll
                for (uint32_t j = 0; j < 4u; ++j)
                    if (q4 + j < n)
                        stg[min(base + q4 + j, cap)] = cb[16u * b + q4 + j];
            }
        }
        // (a packed bucket past nb reads some other LDS word as its slot
        // base: the slot is clamped and the hole it leaves is reported)
        LPROF(1);   // (tags and carried words issued; the placement next)
        auto place = [&](auto ragged) {
            // every slot base of the thread's packets is read before any
            // stage write: a read after a write to the same LDS is ordered
            // behind it, one round trip each
            // (two groups at a time: registers)
#pragma unroll
            for (uint32_t k0 = 0; k0 < kG; k0 += 2u) {
            uint32_t slot[2][8];
#pragma unroll
            for (uint32_t k = k0; k < k0 + 2u; ++k) {
                const uint32_t o8 = 8u * (k * kLineBlock + t);
                // chunks are multiples of 8 packets (clamped: groups past a short span)
                const uint32_t cc = min(o8 >> P.cshift, ncs - 1u);
#pragma unroll
                for (uint32_t j = 0; j < 8u; ++j) {
                    const uint32_t w = (pk[k][j >> 1] >> (16u * (j & 1u))) & 0xffffu;
                    uint32_t b, rk;
                    if (kPacked) {
                        b = w >> P.cshift;
                        rk = w & ((1u << P.cshift) - 1u);
                    } else {
                        b = bucket_of((int16_t)((qk[k][j >> 1] >> (16u * (j & 1u))) & 0xffffu),
                                      P.nq);
                        rk = w;
                    }
                    slot[k - k0][j] = tab[__umul24(b, rs) + cc] + rk;
                }
            }
#pragma unroll
            for (uint32_t k = k0; k < k0 + 2u; ++k) {
                const uint32_t o8 = 8u * (k * kLineBlock + t);
                const uint32_t id = p0 + o8;
#pragma unroll
                for (uint32_t j = 0; j < 8u; ++j)
                    if (!decltype(ragged)::value || o8 + j < len)
                        stg[min(slot[k - k0][j], cap)] = id + j;
            }
            }
        };
        if (len == line_span_max(kG))   // a whole span of the largest size: no lane is past it
            place(std::false_type{});
        else
            place(std::true_type{});
        LPROF(2);
        // the next span's streams and prefixes (issued in (b)) have arrived;
        // waiting here, before this span's list stores, keeps those stores
        // out of the next wait (vmcnt counts loads and stores in one queue).
        // Wave 0 then lays the next span out into set s ^ 1 from its
        // prefixes (no one reads that set in this span), so after the barrier
        // every thread can write the next span's table during the copy-out
        __builtin_amdgcn_s_waitcnt(kWaitVm0);
        if (!last && wave == 0)
            layout(g + 1u, s ^ 1u);
        __syncthreads();
        LPROF(3);
        // (c) copy-out, a quad per thread: whole lines as 16-byte non-temporal
        // stores; the bucket's last line, if the span ends inside it, is
        // carried (unless the range ends here); partial lines word by word
        // One store site for both line modes, its cache policy a template
        // argument: the mode, policy and range branches of each quad were a
        // chain of a dozen scalar and exec branches a turn.
        auto copy_quad = [&](uint32_t v, uint32_t tag, uint32_t gl, const u32x4 &e) {
            const uint32_t mode = tag >> 30;
            const uint32_t a0 = 16u * gl + 4u * (v & 3u);
            bool go = mode == 0u;
            if (mode == 2u) {
                // a partial line (a range's first or last line of a bucket):
                // its quads inside [cs, ve) still leave as one 16-byte store;
                // a quad the bounds cut is left to the cut pass below (word
                // stores for every quad of such lines tripled the scatter's
                // store instructions at 256 buckets)
                const uint32_t b = tag & 0xffffu;
                go = a0 >= cs[b] && a0 + 4u <= ve[b];
            }
            if (!go)
                return;
            const uint32_t d = a0 - ph;
            if (d + 4u <= P.n && d + 4u > d) {
                if (__builtin_expect(P.merge != 0u, 0) && mode == 2u)
                    line_store4<0>(lout, d, e);   // plain: the line's other part meets it in L2
                else
                    line_store4<kNtAux>(lout, d, e);
                wrote += 4u;
                wsum += e.x + e.y + e.z + e.w;
            } else {
                report_fault(P.fault, YRSS_FAULT_LIST_RANGE, YRSS_K_SCATTER, g, d);
            }
        };
        // kCopyQ quads a turn, all loaded before any is stored (an
        // 8192-packet span's lines fit one turn up to ~128 buckets); the next
        // span's table first (tab is read only in (b), before the barrier)
        constexpr uint32_t kCopyQ = 5u, nct = kLineBlock;
        if (!last)
            write_tab(s ^ 1u);
        LPROF(6);
        for (uint32_t v0 = t; v0 < 4u * L; v0 += kCopyQ * nct) {
            uint32_t tg[kCopyQ], gl[kCopyQ];
            u32x4 eq[kCopyQ];
#pragma unroll
            for (uint32_t i = 0; i < kCopyQ; ++i) {
                const uint32_t v = v0 + i * nct;
                tg[i] = 1u << 30;   // mode 1: nothing to store
                gl[i] = 0u;
                eq[i] = u32x4{0u, 0u, 0u, 0u};
                if (v < 4u * L) {
                    tg[i] = ltag[v >> 2];
                    gl[i] = lgl[v >> 2];
                    eq[i] = reinterpret_cast<const u32x4 *>(stg)[v];
                }
            }
#pragma unroll
            for (uint32_t i = 0; i < kCopyQ; ++i)
                copy_quad(v0 + i * nct, tg[i], gl[i], eq[i]);
        }
        // The cut quads of partial lines: per bucket at most two, the quad
        // holding its first valid position cs (when unaligned) and the one
        // holding its end ve (when unaligned and the line leaves now, i.e.
        // the range ends here).  A thread per (bucket, quad, word), one word
        // a lane, from the stage: a wave-instruction stores 64 such words
        // where the copy-out's per-quad word stores cost four
        // wave-instructions for every turn that held one
        // (only the range's last span can cut an end; a start is cut only
        // while some bucket's first valid position is off a quad: layout
        // records that, so a middle span usually skips the pass)
        const uint32_t ncut = last || misc[6u + s] ? 8u * nb : 0u;
        for (uint32_t e = tr; e < ncut; e += kLineBlock) {
            const uint32_t b = e >> 3, k = (e >> 2) & 1u, j = e & 3u;
            const uint32_t v0 = cs[b], e1 = ve[b];
            const uint32_t qb = (k ? e1 : v0) & ~3u, a = qb + j;
            bool go = a >= v0 && a < e1 && ((k ? e1 : v0) & 3u) != 0u;
            if (k == 0u)   // the first cut quad's line leaves now unless carried
                go = go && !(!last && (v0 >> 4) == (e1 >> 4) && (e1 & 15u) != 0u);
            else           // the end's line leaves now only at the range's end;
                           // a quad holding both bounds, v0 unaligned, is k = 0's
                go = go && last && !(qb == (v0 & ~3u) && (v0 & 3u) != 0u);
            if (go) {
                const uint32_t w = stg[min(so[b] + a, cap)], d = a - ph;
                if (d < P.n) {
                    if (P.merge)
                        line_store1<0>(lout, d, w);
                    else
                        line_store1<kNtAux>(lout, d, w);
                    ++wrote;
                    wsum += w;
                } else {
                    report_fault(P.fault, YRSS_FAULT_LIST_RANGE, YRSS_K_SCATTER, g, d);
                }
            }
        }
        LPROF(4);
        // (d) carry the unfinished last lines
        if (!last) {
            // a quad a thread: a 16-byte copy where the stage slots are
            // aligned (the words past the end carry nothing the next span
            // reads), else word by word
            for (uint32_t e = tr; e < 4u * nb; e += kLineBlock) {
                const uint32_t b = e >> 2, q4 = 4u * (e & 3u);
                const uint32_t e1 = ve[b], nv = max(cs[b], e1 & ~15u);
                const uint32_t n = e1 - nv, base = so[b] + nv;
                if (q4 >= n)
                    continue;
                if (((base + q4) & 3u) == 0u && base + q4 <= cap) {
                    reinterpret_cast<u32x4 *>(cb)[4u * b + (q4 >> 2)] =
                        reinterpret_cast<const u32x4 *>(stg)[(base + q4) >> 2];
                } else {
#pragma unroll
                    for (uint32_t j = 0; j < 4u; ++j)
                        if (q4 + j < n)
                            cb[16u * b + q4 + j] = stg[min(base + q4 + j, cap)];
                }
            }
            // the next span's placement overwrites the stage and tags read above
            __syncthreads();
        }
        LPROF(5);
    };
    for (uint32_t g = g0; g < g1; g += 2u) {
        span(g, 0u, pkA, qkA, pkB, qkB);
        if (g + 1u < g1)
            span(g + 1u, 1u, pkB, qkB, pkA, qkA);
    }
    // every packet of the range left exactly once
    wrote = __shfl(wave_incl_scan(wrote, lane), kWave - 1, kWave);
    wsum = __shfl(wave_incl_scan(wsum, lane), kWave - 1, kWave);
    if (lane == 0) {
        atomicAdd(&misc[3], wrote);
        atomicAdd(&misc[1], wsum);
    }
    __syncthreads();
    if (t == 0) {
        const uint64_t a = (uint64_t)g0 * P.seg, e = span_end(g1 - 1u);
        const uint32_t want = (uint32_t)(e - a);
        const uint32_t want_sum = (uint32_t)((e - a) * (a + e - 1u) / 2u);
        if (misc[3] != want)
            report_fault(P.fault, YRSS_FAULT_COUNT_MISMATCH, YRSS_K_SCATTER, g0, misc[3]);
        else if (misc[1] != want_sum)
            report_fault(P.fault, YRSS_FAULT_STAGE, YRSS_K_SCATTER, g0, misc[1]);
    }
}

// ---------------------------------------------------------------------------
// ff_rss_check (ff_dpdk_if.c:1904-1940) in batch: the connect-side RSS check
// F-Stack runs per candidate lport in in_pcbconnect_setup (in_pcb.c:1131-1170).
// The tuple is hashed in its raw stored (network-order) byte order, unlike
// toeplitz_dispatch's ntohl'd tuple.  One lane per tuple; 12 LDS lookups.
// ---------------------------------------------------------------------------
struct RssCheckParams {
    const yrss_rss_tuple *tuples;   // batch mode
    uint8_t *ok;
    uint32_t *hash;
    uint32_t *bitmap;               // sweep mode: 2048 words
    uint32_t n;
    uint32_t fixed[3];              // sweep mode: saddr, daddr, sport (as stored)
    uint32_t nq;
    uint32_t mask;                  // (uint32_t)(int)(reta_size - 1)
    uint32_t queueid;
    uint32_t sweep;
    uint32_t kwin[96];
};

__device__ __forceinline__ uint32_t hash_raw12(const uint32_t *tbl, uint32_t w0, uint32_t w1,
                                               uint32_t w2)
{
    uint32_t h = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        h ^= tbl[(0 + b) * 256 + ((w0 >> (8 * b)) & 0xffu)];
        h ^= tbl[(4 + b) * 256 + ((w1 >> (8 * b)) & 0xffu)];
        h ^= tbl[(8 + b) * 256 + ((w2 >> (8 * b)) & 0xffu)];
    }
    return h;
}

__global__ __launch_bounds__(256) void yrss_rss_check(RssCheckParams P)
{
    __shared__ uint32_t tbl[12 * 256];
    for (uint32_t e = threadIdx.x; e < 12u * 256u; e += 256u) {
        const uint32_t jt = e >> 8, v = e & 255u;
        uint32_t acc = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b)
            acc ^= (v & (0x80u >> b)) ? P.kwin[8 * jt + b] : 0u;
        tbl[e] = acc;
    }
    __syncthreads();
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    uint32_t w0, w1, w2;
    if (P.sweep) {
        // stored lport value p occupies tuple bytes 10..11 as its little-endian image
        w0 = P.fixed[0];
        w1 = P.fixed[1];
        w2 = (P.fixed[2] & 0xffffu) | ((i & 0xffffu) << 16);
    } else {
        const uint32_t k = i < P.n ? i : (P.n ? P.n - 1u : 0u);
        const uint32_t *t = reinterpret_cast<const uint32_t *>(P.tuples + k);
        w0 = t[0];
        w1 = t[1];
        w2 = t[2];
    }
    const uint32_t h = hash_raw12(tbl, w0, w1, w2);
    const bool ok = P.nq <= 1u || ((h & P.mask) % P.nq) == P.queueid;
    if (P.sweep) {
        const uint64_t m = __ballot(ok);
        const uint32_t lane = lane_id();
        if (lane == 0)
            P.bitmap[i >> 5] = (uint32_t)m;
        else if (lane == 32)
            P.bitmap[i >> 5] = (uint32_t)(m >> 32);
    } else if (i < P.n) {
        P.ok[i] = ok ? 1u : 0u;
        if (P.hash)
            P.hash[i] = h;
    }
}

// ---------------------------------------------------------------------------
// Zero-copy gather: header windows straight out of host-resident rte_mbufs.
// Four lanes per packet: one wave-instruction reads the first 64 bytes of 16
// mbuf headers (one 64-byte PCIe read each), the quad exchanges buf_addr /
// data_off / data_len by shuffles, then reads the packet's header window the
// same way (rte_pktmbuf_mtod, rte_mbuf.h:1620) and stores it to HBM in the
// yrss_dispatch_dev layout (stride 80).
// ---------------------------------------------------------------------------
struct HostRange {
    uint64_t lo, hi;      // host virtual range [lo, hi)
    int64_t delta;        // device address = host address + delta
};

struct GatherParams {
    const uint64_t *ptrs;       // mbuf (or frame data) pointers, device-visible
    const uint16_t *lens;       // frames mode: data_len per frame, device-visible
    uint8_t *win;               // n x 80
    uint16_t *len;
    uint32_t *fault;            // set when a pointer is outside every range
    const uint32_t *hash;       // write-back mode: hash per packet
    uint32_t n;
    uint32_t nranges;
    uint32_t off_buf_addr, off_data_off, off_data_len, off_hash_rss;
    uint32_t frames;            // 1: ptrs are frame data pointers, lens given
    HostRange ranges[YRSS_MAX_HOST_RANGES];
};

__device__ __forceinline__ bool host_xlate(const GatherParams &G, uint64_t a, uint32_t bytes,
                                           int64_t *delta)
{
    for (uint32_t r = 0; r < G.nranges; ++r)
        if (a >= G.ranges[r].lo && a + bytes <= G.ranges[r].hi) {
            *delta = G.ranges[r].delta;
            return true;
        }
    return false;
}

// 16 bytes from host memory at any alignment (DPDK data is normally 64-byte
// aligned; rte_pktmbuf_adj can leave it anywhere).
__device__ __forceinline__ u32x4 host_load16(uint64_t a)
{
    if ((a & 15u) == 0)
        return *reinterpret_cast<const u32x4 *>(a);
    u32x4 v;
    if ((a & 3u) == 0) {
        const uint32_t *p = reinterpret_cast<const uint32_t *>(a);
        v.x = p[0]; v.y = p[1]; v.z = p[2]; v.w = p[3];
        return v;
    }
    const uint8_t *b = reinterpret_cast<const uint8_t *>(a);
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        w[k] = b[4 * k] | (b[4 * k + 1] << 8) | (b[4 * k + 2] << 16) | ((uint32_t)b[4 * k + 3] << 24);
    v.x = w[0]; v.y = w[1]; v.z = w[2]; v.w = w[3];
    return v;
}

__device__ __forceinline__ uint32_t pick_word(const u32x4 &v, uint32_t k)
{
    return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}

// dword at byte offset o (4-aligned, < 64) of the quad's 64-byte header
__device__ __forceinline__ uint32_t quad_word(const u32x4 &hv, uint32_t lane, uint32_t o)
{
    return __shfl(pick_word(hv, (o >> 2) & 3u), (int)((lane & ~3u) | (o >> 4)), kWave);
}

// Windows of the calling wave's packets (4 lanes per packet, 16 packets per
// wave-iteration): the mbuf header (or the frame pointer/length pair) and the
// first 80 bytes of data, read from registered host memory, into G.win at
// stride 80 and G.len.  kB iterations run in lockstep phases (pointers, then
// headers, then data), so a wave has kB x 16 packets' PCIe reads in flight
// per dependent step instead of 16.
// The per-call pointers of a gather, apart from the range table and the mbuf
// layout (GatherParams), so a persistent caller can vary them per burst
// without copying the table.
struct GatherIO {
    const uint64_t *ptrs;
    const uint16_t *lens;
    uint8_t *win;
    uint16_t *len;
    uint32_t *fault;
    uint32_t n;
    uint32_t frames;     // 1: ptrs are frame data pointers, lens given
};

__device__ __forceinline__ GatherIO gather_io(const GatherParams &G)
{
    return GatherIO{G.ptrs, G.lens, G.win, G.len, G.fault, G.n, G.frames};
}

template <int kB>
__device__ __forceinline__ void gather_quads(const GatherParams &G, const GatherIO &io,
                                             uint32_t wave, uint32_t nwaves, uint32_t lane)
{
    const uint32_t c = lane & 3u;
    for (uint32_t p0 = wave * 16u * kB; p0 < io.n; p0 += nwaves * 16u * kB) {
        uint32_t idx[kB], L[kB];
        uint64_t m[kB], data[kB];
        bool ok_m[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            idx[k] = p0 + 16u * k + (lane >> 2);
            m[k] = idx[k] < io.n ? io.ptrs[idx[k]] : 0u;
            L[k] = (io.frames && idx[k] < io.n) ? io.lens[idx[k]] : 0u;
        }
        if (io.frames) {
            // frames mode: the host already knows data pointer and data_len
#pragma unroll
            for (int k = 0; k < kB; ++k) {
                data[k] = m[k];
                ok_m[k] = idx[k] < io.n;
            }
        } else {
            u32x4 hv[kB];
            int64_t dm[kB];
#pragma unroll
            for (int k = 0; k < kB; ++k) {
                dm[k] = 0;
                ok_m[k] = idx[k] < io.n && host_xlate(G, m[k], 64u, &dm[k]);
                hv[k] = u32x4{0u, 0u, 0u, 0u};
                if (ok_m[k])
                    hv[k] = host_load16(m[k] + dm[k] + 16u * c);
            }
            const uint32_t ob = G.off_buf_addr, od = G.off_data_off, ol = G.off_data_len;
#pragma unroll
            for (int k = 0; k < kB; ++k) {
                const uint64_t buf = (uint64_t)quad_word(hv[k], lane, ob) |
                                     ((uint64_t)quad_word(hv[k], lane, ob + 4u) << 32);
                const uint32_t doff =
                    (quad_word(hv[k], lane, od & ~3u) >> (8u * (od & 3u))) & 0xffffu;
                L[k] = (quad_word(hv[k], lane, ol & ~3u) >> (8u * (ol & 3u))) & 0xffffu;
                data[k] = buf + doff;
            }
        }
        u32x4 w[kB], t[kB];
        bool ok_d[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const uint32_t need = (min(L[k], (uint32_t)YRSS_WIN_FULL) + 15u) & ~15u;
            int64_t dd = 0;
            ok_d[k] = ok_m[k] && (need == 0 || host_xlate(G, data[k], need, &dd));
            w[k] = u32x4{0u, 0u, 0u, 0u};
            t[k] = u32x4{0u, 0u, 0u, 0u};
            if (ok_d[k] && 16u * c < need)
                w[k] = host_load16(data[k] + dd + 16u * c);
            if (ok_d[k] && c == 0 && need > 64u)
                t[k] = host_load16(data[k] + dd + 64u);
        }
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            if (idx[k] >= io.n)
                continue;
            uint8_t *dst = io.win + (size_t)idx[k] * YRSS_WIN_FULL;
            *reinterpret_cast<u32x4 *>(dst + 16u * c) = w[k];
            if (c == 0) {
                *reinterpret_cast<u32x4 *>(dst + 64u) = t[k];
                io.len[idx[k]] = (uint16_t)L[k];
                if (!ok_d[k])   // plain store: the word may live in host memory
                    __hip_atomic_store(io.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

__global__ __launch_bounds__(256) void yrss_gather_zc(GatherParams G)
{
    const uint32_t wave = (blockIdx.x * 256u + threadIdx.x) / kWave;
    gather_quads<1>(G, gather_io(G), wave, gridDim.x * (256u / kWave), lane_id());
}

// hash.rss write-back straight into the host mbufs (YRSS_F_WRITE_RSS)
__global__ __launch_bounds__(256) void yrss_writeback_zc(GatherParams G)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= G.n)
        return;
    const uint64_t m = G.ptrs[i];
    int64_t dm = 0;
    if (host_xlate(G, m, G.off_hash_rss + 4u, &dm))
        *reinterpret_cast<uint32_t *>(m + dm + G.off_hash_rss) = G.hash[i];
}

// ---------------------------------------------------------------------------
// Small host bursts (n <= 4096, nb <= 64) in ONE launch of ONE workgroup.
// The host-resident entry points at F-Stack's burst sizes (32 at
// ff_dpdk_if.c:83, 1024 in BASELINE) were bound by per-call HIP overhead:
// memset + gather + parse + scan + scatter + four D2H copies = ten queue
// operations, 39-62 us a burst.  Here 16 waves do everything:
//   gather   (zero-copy modes) mbuf headers and windows from registered host
//            memory into device scratch (gather_quads, each wave its own
//            tiles, pointer / header / data reads in lockstep rounds);
//   parse    each wave loads all its (up to four) 64-packet tiles, then runs
//            them through the same process_tile() as yrss_parse_hash
//            (per-tile bucket counts and per-packet ranks in LDS, outputs
//            kept in the wave's LDS buffer);
//   lists    per-bucket prefix over the tiles in LDS, then every packet's
//            list slot = start[b] + prefix[tile][b] + rank: the same stable
//            FIFO lists as parse + scan + scatter;
//   outputs  straight into host-visible memory (the caller's registered
//            arrays or the context's pinned staging), so no copy follows.
// A multi-workgroup variant (one tile per wave, last-arriver ticket for the
// lists) was slower at every burst size measured: 21 vs 16 us at 32 packets,
// 34 vs 33 at 1024 (profiles/r01_v11_small_burst.log).
// ---------------------------------------------------------------------------
constexpr int kSmallBlock = 1024;
constexpr uint32_t kSmallWaves = kSmallBlock / kWave;          // 16
constexpr uint32_t kSmallTiles = kSmallWaves * kOutTiles;      // 64
constexpr uint32_t kSmallMaxPkts = kSmallTiles * kTile;        // 4096
constexpr uint32_t kSmallMaxNb = kWave;                        // one lane per bucket

struct SmallParams {
    ParseParams P;       // win/len: windows to parse; q/hash/filter: host-visible outputs
    GatherParams G;      // gather: source pointers; G.win/G.len = P.win/P.len (scratch)
    uint32_t *qidx;      // host-visible, or null
    uint32_t *qstart;    // host-visible [nb + 1], or null
    uint32_t gather;     // 1: gather the windows first (zero-copy modes)
    uint32_t writeback;  // 1: store hash.rss into each mbuf (YRSS_F_WRITE_RSS)
    uint64_t *done;      // host-coherent completion word, or null
    uint64_t seq;        // stored into *done once every output is visible to the host
};

__host__ __device__ inline size_t small_lds(uint32_t nb, bool filter)
{
    return kTblBytes + kSmallWaves * (kStageBytes + kOutBytes) +
           (size_t)(kSmallTiles * nb + kSmallMaxNb) * sizeof(uint32_t) +
           (filter ? kKniWords * sizeof(uint32_t) : 0u);
}

// LDS carve-up shared by the one-shot kernel and the worker.
struct SmallLds {
    uint32_t *tbl;
    u32x4 *stage;
    uint32_t *oh;
    uint16_t *oq;
    int8_t *of;
    uint16_t *orank;
    uint32_t *cnt;
    uint32_t *start;
    uint32_t *kni;
};

__device__ __forceinline__ SmallLds small_carve(uint8_t *smem, uint32_t wave, uint32_t nb)
{
    SmallLds L;
    L.tbl = reinterpret_cast<uint32_t *>(smem);
    L.stage = reinterpret_cast<u32x4 *>(smem + kTblBytes + wave * kStageBytes);
    uint8_t *out_w = smem + kTblBytes + kSmallWaves * kStageBytes + wave * kOutBytes;
    L.oh = reinterpret_cast<uint32_t *>(out_w);
    L.oq = reinterpret_cast<uint16_t *>(out_w + kOutTiles * kTile * 4);
    L.of = reinterpret_cast<int8_t *>(out_w + kOutTiles * kTile * 6);
    L.orank = reinterpret_cast<uint16_t *>(out_w + kOutTiles * kTile * 7);
    L.cnt = reinterpret_cast<uint32_t *>(smem + kTblBytes +
                                         kSmallWaves * (kStageBytes + kOutBytes));
    L.start = L.cnt + kSmallTiles * nb;
    L.kni = L.start + kSmallMaxNb;
    return L;
}

// Byte tables (and KNI bitmaps) for the workgroup; the caller synchronises.
template <bool kFilter>
__device__ __forceinline__ void small_tables(const ParseParams &P, const SmallLds &L)
{
    build_key_tables(L.tbl, P.kwin, threadIdx.x, kSmallBlock);
    if (kFilter)
        for (uint32_t e = threadIdx.x; e < (uint32_t)kKniWords; e += kSmallBlock)
            L.kni[e] = P.kni_enable ? P.kni_bm[e] : 0u;
}

// One burst through one workgroup, tables already in LDS: gather (zero-copy
// modes), parse, per-bucket FIFO lists, outputs to host-visible memory.
// Per-burst outputs and switches of small_burst_body.
struct BurstIO {
    uint32_t *qidx;      // host-visible, or null
    uint32_t *qstart;    // host-visible [nb + 1], or null
    uint32_t gather;     // 1: gather the windows first (zero-copy modes)
    uint32_t writeback;  // 1: store hash.rss into each mbuf (YRSS_F_WRITE_RSS)
    uint64_t *done;      // host-coherent completion word, or null
    uint64_t seq;        // stored into *done once every output is visible to the host
};

template <bool kFilter, uint32_t kTW = kOutTiles>   // kTW: tiles per wave (n <= kTW * 1024)
__device__ void small_burst_body(const ParseParams &P, const GatherParams &G, const GatherIO &gio,
                                 const BurstIO &S, const SmallLds &L, uint32_t wave,
                                 uint32_t lane)
{
    // wave w owns tiles w, w + 16, w + 32, w + 48: with 4 lockstep rounds of
    // 16 packets, gather_quads' wave-iteration p0 = 64 (w + 16 j) is tile j's
    if (S.gather)
        gather_quads<4>(G, gio, wave, kSmallWaves, lane);
    for (uint32_t e = threadIdx.x; e < kSmallTiles * P.nb; e += kSmallBlock)
        L.cnt[e] = 0;
    // also orders the gathered windows (global scratch written by this
    // workgroup) before the parse reads them
    __syncthreads();

    const uint32_t ntiles = (P.n + kTile - 1) / kTile;
    // all of the wave's tiles are loaded before the first is parsed: the
    // windows may sit in host memory, one PCIe round trip for all of them
    u32x4 r[kTW][4];
    uint32_t Ln[kTW];
#pragma unroll
    for (uint32_t j = 0; j < kTW; ++j) {
        const uint32_t t = min(wave + j * kSmallWaves, ntiles - 1u);
        load_tile<false>(P, t * kTile, P.n, lane, r[j], Ln[j]);
    }
#pragma unroll
    for (uint32_t j = 0; j < kTW; ++j) {
        const uint32_t t = wave + j * kSmallWaves;
        if (t >= ntiles)
            break;
        process_tile<2, kFilter>(P, L.tbl, L.kni, L.stage, L.cnt + t * P.nb,
                                 OutSlot{L.oq + j * kTile, L.oh + j * kTile, L.of + j * kTile,
                                         L.orank + j * kTile},
                                 t * kTile, P.n, lane, r[j], Ln[j]);
    }
    __syncthreads();
    // per bucket: exclusive prefix over the tiles (in place) and the total
    if (threadIdx.x < P.nb) {
        const uint32_t b = threadIdx.x;
        uint32_t run = 0;
        for (uint32_t t = 0; t < ntiles; ++t) {
            const uint32_t v = L.cnt[t * P.nb + b];
            L.cnt[t * P.nb + b] = run;
            run += v;
        }
        L.start[b] = run;
    }
    __syncthreads();
    if (wave == 0) {
        const uint32_t tot = lane < P.nb ? L.start[lane] : 0u;
        const uint32_t x = wave_incl_scan(tot, lane);
        if (lane < P.nb) {
            L.start[lane] = x - tot;
            if (S.qstart)
                S.qstart[lane] = x - tot;
        }
        if (lane == kWave - 1 && S.qstart)
            S.qstart[P.nb] = x;
    }
    __syncthreads();
    for (uint32_t j = 0; j < kTW; ++j) {
        const uint32_t t = wave + j * kSmallWaves;
        if (t >= ntiles)
            break;
        flush_out<kFilter>(P, L.oq + j * kTile, L.oh + j * kTile, L.of + j * kTile,
                           L.orank + j * kTile, t * kTile, 1u, lane);
        const uint32_t pkt = t * kTile + lane;
        if (pkt < P.n) {
            if (S.qidx) {
                const uint32_t b = bucket_of((int16_t)L.oq[j * kTile + lane], P.nq);
                const uint32_t d = L.start[b] + L.cnt[t * P.nb + b] + L.orank[j * kTile + lane];
                if (d < P.n)
                    S.qidx[d] = pkt;
                else
                    report_fault(P.fault, YRSS_FAULT_LIST_RANGE, YRSS_K_BURST, pkt, d);
            }
            if (S.writeback) {
                const uint64_t m = gio.ptrs[pkt];
                int64_t dm = 0;
                if (host_xlate(G, m, G.off_hash_rss + 4u, &dm))
                    *reinterpret_cast<uint32_t *>(m + dm + G.off_hash_rss) =
                        L.oh[j * kTile + lane];
            }
        }
    }
}

template <bool kFilter>
__global__ __launch_bounds__(kSmallBlock) void yrss_burst_small(SmallParams S)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const SmallLds L = small_carve(smem, wave, S.P.nb);
    small_tables<kFilter>(S.P, L);
    small_burst_body<kFilter>(S.P, S.G, gather_io(S.G),
                              BurstIO{S.qidx, S.qstart, S.gather, S.writeback}, L, wave,
                              lane_id());
    if (S.done) {
        // the host spins on this word instead of a stream synchronisation:
        // every wave's stores drained, one system-scope release, then the word
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(S.done, S.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ---------------------------------------------------------------------------
// Persistent burst worker (yrss_worker_*): no launch and no stream
// synchronisation per burst.  The host writes a burst's mbuf pointers into a
// slot of a ring in host-coherent pinned memory and publishes its ticket in
// the slot's seq word; workgroup b of this kernel owns tickets b+1, b+1+B,
// ... (B workgroups; slot = ticket mod nslots, nslots a multiple of B), polls
// the seq word of its next ticket, runs the burst through small_burst_body()
// (tables stay in LDS across bursts), writes q / hash / lists to the output
// addresses the slot names (the caller's registered arrays or the slot's
// pinned staging) and publishes the ticket in done[slot], a separate
// GPU-written array.  Every workgroup leaves when the host sets the stop word,
// after the whole ring saw no submit for idle_ticks, or after life_ticks in
// total, storing the ticket it would have served next and counting itself in
// WorkerCtl::exited; the host's next submit or poll then stops the rest of
// the launch and relaunches.
// Protocol (host-coherent memory, system scope): the host writes ptrs / n /
// flags / output addresses, then seq with release; the GPU polls seq relaxed,
// then acquires and reads the addresses (unless its LDS cache has them).
// The GPU drains every wave's output stores (vmcnt(0) + barrier), releases
// at system scope, then writes done; the host reads done with acquire.
// ---------------------------------------------------------------------------
constexpr uint32_t kWorkerMaxBurst = YRSS_WORKER_MAX_BURST;   // 16 tiles: one per wave

// Written by the host only, so its submit stores stay cache hits; the GPU
// answers in a separate done array (WorkerParams::done).
struct alignas(64) WorkerSlot {
    uint64_t seq;        // ticket, written last (release)
    uint32_t n;          // packets (written before seq; read with it, one 16-B load)
    uint32_t flags;      // YRSS_F_WRITE_RSS | kWorkerFrames
    // device addresses of q, hash, qidx, qstart (read after the acquire): the
    // caller's own arrays when they lie in registered memory (no copy at
    // poll), else the slot's staging; 0 = not wanted
    uint64_t out[4];
    uint64_t win;        // windows form: device address of window 0 (stride below)
    uint32_t stride;
    uint32_t pad_;
};
// done[slot] = ticket | kWorkerFault when a pointer was outside every range,
// | kWorkerGuard when a list guard of this burst fired (its record is then in
// the slot's entry of WorkerParams::srec).  The fault travels with the burst:
// bursts of other workgroups in flight at the same time never see it.
// Consecutive slots share a line, so a host polling in ticket order misses
// once per eight bursts instead of once per burst.
constexpr uint64_t kWorkerFault = 1ull << 63;
constexpr uint64_t kWorkerGuard = 1ull << 62;
constexpr uint64_t kWorkerFlags = kWorkerFault | kWorkerGuard;
// flags bit: the slot's output addresses equal those of its previous burst, so
// a workgroup that cached them may skip reading them (one PCIe round trip)
constexpr uint32_t kWorkerSameOut = 1u << 17;
constexpr uint32_t kWorkerOutCache = 32;   // cached slots per workgroup (LDS)
constexpr uint32_t kWorkerFrames = 1u << 16;   // slot holds (data, data_len) pairs
constexpr uint32_t kWorkerWindows = 1u << 18;  // slot names contiguous windows (win, stride)
static_assert(sizeof(WorkerSlot) == 64, "one line per slot header");

// Launch control, host-coherent.  Line 0 is written by the host only (so
// the host's per-submit store stays a cache hit), line 1 by the GPU only.
struct alignas(64) WorkerCtl {
    uint32_t stop;       // host: leave now
    uint32_t pad0_;
    uint64_t pub;        // host: latest published ticket (ring activity)
    uint32_t pad1_[12];
    uint32_t exited;     // GPU: workgroups of this launch that left
    uint32_t pad2_[15];
};
static_assert(sizeof(WorkerCtl) == 128, "two lines");

struct WorkerParams {
    ParseParams P;       // configuration (per-burst fields set in the kernel)
    GatherParams G;      // range table and mbuf layout
    WorkerSlot *slots;   // [nslots] host-coherent, host-written
    uint64_t *done;      // [nslots] host-coherent, GPU-written
    uint32_t *fault;     // [nblocks] device: gather fault of the current burst
    uint32_t *brec;      // [nblocks][4] device: guard record of the current burst
    uint32_t *srec;      // [nslots][4] host-coherent: guard record of the slot's burst
    uint64_t inject;     // -DYRSS_TEST_HOOKS builds only: ticket whose burst fires a guard
    uint64_t *ptrs;      // [nslots][kWorkerMaxBurst] pinned: mbuf or frame data pointers
    uint16_t *lens;      // [nslots][kWorkerMaxBurst] pinned: frame data_len (frames mode)
    uint8_t *win;        // device scratch [nblocks][kWorkerMaxBurst * 80]
    uint16_t *len;       // device scratch [nblocks][kWorkerMaxBurst]
    uint64_t *next;      // host-coherent [nblocks]: ticket to serve next (resume)
    WorkerCtl *wctl;     // host-coherent launch control
    uint32_t nslots;
    uint64_t idle_ticks; // s_memrealtime ticks (100 MHz)
    uint64_t life_ticks;
    uint32_t poll_sleep; // s_sleep(2) units between two polls of a slot
};

// small_burst_body's LDS, then 64 B of control words, then the output-address
// cache: kWorkerOutCache slots x 4 addresses and one valid word per slot
size_t worker_lds(uint32_t nb)
{
    return small_lds(nb, false) + 64u + kWorkerOutCache * (32u + 4u);
}

__global__ __launch_bounds__(kSmallBlock) void yrss_burst_worker(WorkerParams W)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint32_t lane = lane_id();
    const SmallLds L = small_carve(smem, wave, W.P.nb);
    uint32_t *ctl = reinterpret_cast<uint32_t *>(smem + small_lds(W.P.nb, false));
    uint64_t *ocache = reinterpret_cast<uint64_t *>(ctl + 16);
    uint32_t *ovalid = reinterpret_cast<uint32_t *>(ocache + 4 * kWorkerOutCache);
    // slots of this workgroup: slot of ticket t is t mod nslots, and the
    // workgroup's tickets are b+1 + kB, so its slots are (b+1 + kB) mod nslots
    const uint32_t my_slots = W.nslots / gridDim.x;
    for (uint32_t i = threadIdx.x; i < kWorkerOutCache; i += blockDim.x)
        ovalid[i] = 0u;
    small_tables<false>(W.P, L);

    uint64_t t = __hip_atomic_load(W.next + blockIdx.x, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t t_begin = wall_clock64();
    uint64_t t_last = t_begin;
    uint64_t pub_seen = 0;   // thread 0 only: ring activity at the last idle check
    if (threadIdx.x == 0)
        pub_seen = __hip_atomic_load(&W.wctl->pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (;;) {
        const uint32_t si = (uint32_t)(t % W.nslots);
        WorkerSlot *sl = W.slots + si;
        if (threadIdx.x == 0) {
            uint32_t go = 0;   // 1: a burst, 2: leave
            for (;;) {
                // seq, n and flags in one 16-byte read: the host writes n and
                // flags before seq, so a new seq comes with its n and flags
                const u32x4 hd = *reinterpret_cast<const volatile u32x4 *>(sl);
                if ((((uint64_t)hd.y << 32) | hd.x) == t) {
                    ctl[1] = hd.z;
                    ctl[2] = hd.w;
                    go = 1;
                    break;
                }
                const uint64_t now = wall_clock64();
                if (__hip_atomic_load(&W.wctl->stop, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM) ||
                    now - t_begin > W.life_ticks) {
                    go = 2;
                    break;
                }
                if (now - t_last > W.idle_ticks) {
                    // idle is collective: leave only when the whole ring saw no
                    // submit for an idle period, so at low rates (fewer than B
                    // bursts per idle period) no workgroup leaves while others
                    // keep serving and strands its tickets
                    const uint64_t pub = __hip_atomic_load(&W.wctl->pub, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_SYSTEM);
                    if (pub == pub_seen) {
                        go = 2;
                        break;
                    }
                    pub_seen = pub;
                    t_last = now;
                }
                // each poll is a PCIe read: many resident workgroups polling
                // back to back compete with the bursts' own reads
                for (uint32_t z = 0; z < W.poll_sleep; ++z)
                    __builtin_amdgcn_s_sleep(2);
            }
            if (go == 1) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                __hip_atomic_store(W.fault + blockIdx.x, 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(W.brec + 4u * blockIdx.x, 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                // local index of this slot among the workgroup's slots
                const uint32_t li = si / gridDim.x;
                const bool cacheable = my_slots <= kWorkerOutCache;
                uint64_t o[4];
                if (cacheable && (ctl[2] & kWorkerSameOut) && ovalid[li]) {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        o[k] = ocache[4 * li + k];
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        o[k] = __hip_atomic_load(&sl->out[k], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM);
                    if (cacheable) {
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            ocache[4 * li + k] = o[k];
                        ovalid[li] = 1u;
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    ctl[4 + 2 * k] = (uint32_t)o[k];
                    ctl[5 + 2 * k] = (uint32_t)(o[k] >> 32);
                }
                if (ctl[2] & kWorkerWindows) {
                    const uint64_t wb = __hip_atomic_load(&sl->win, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_SYSTEM);
                    ctl[12] = (uint32_t)wb;
                    ctl[13] = (uint32_t)(wb >> 32);
                    ctl[14] = __hip_atomic_load(&sl->stride, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
            ctl[0] = go;
        }
        __syncthreads();
        if (ctl[0] != 1u)
            break;
        const uint32_t n = min(ctl[1], kWorkerMaxBurst);
        ParseParams P = W.P;
        P.n = n;
        P.fault = W.brec + 4u * blockIdx.x;   // this burst's own record
#ifdef YRSS_TEST_HOOKS   // libyrss_test.so only: the per-burst fault path's test
        if (t == W.inject && threadIdx.x == 0)
            report_fault(P.fault, YRSS_FAULT_LIST_RANGE, YRSS_K_WORKER, (uint32_t)t, 0xdeadu);
#endif
        P.win = W.win + (size_t)blockIdx.x * kWorkerMaxBurst * YRSS_WIN_FULL;
        P.len = W.len + (size_t)blockIdx.x * kWorkerMaxBurst;
        P.stride = YRSS_WIN_FULL;
        auto out_ptr = [&](int k) {
            return (void *)(uintptr_t)(((uint64_t)ctl[5 + 2 * k] << 32) | ctl[4 + 2 * k]);
        };
        P.q = static_cast<int16_t *>(out_ptr(0));
        P.hash = static_cast<uint32_t *>(out_ptr(1));
        P.filter = nullptr;
        P.seg_cnt = nullptr;
        P.rank = nullptr;
        P.out16 = 0;
        const uint32_t frames = (ctl[2] & kWorkerFrames) ? 1u : 0u;
        const bool windows = (ctl[2] & kWorkerWindows) != 0;
        if (windows) {
            // the caller copied the burst's windows contiguously into
            // registered memory: the parse reads them in place, one stretch
            // of host memory, with no pointer reads and no gather
            P.win = reinterpret_cast<const uint8_t *>(((uint64_t)ctl[13] << 32) | ctl[12]);
            P.stride = ctl[14];
            P.len = W.lens + (size_t)si * kWorkerMaxBurst;
        }
        const GatherIO gio{W.ptrs + (size_t)si * kWorkerMaxBurst,
                           W.lens + (size_t)si * kWorkerMaxBurst, const_cast<uint8_t *>(P.win),
                           const_cast<uint16_t *>(P.len), W.fault + blockIdx.x, n, frames};
        if (n) {
            small_burst_body<false, 1>(P, W.G, gio,
                                    BurstIO{static_cast<uint32_t *>(out_ptr(2)),
                                            static_cast<uint32_t *>(out_ptr(3)),
                                            windows ? 0u : 1u,
                                            (!frames && !windows && (ctl[2] & YRSS_F_WRITE_RSS))
                                                ? 1u : 0u},
                                    L, wave, lane);
        } else if (threadIdx.x <= W.P.nb && out_ptr(3)) {
            static_cast<uint32_t *>(out_ptr(3))[threadIdx.x] = 0u;
        }
        // every wave's output stores drained, then one system-scope release
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t f = __hip_atomic_load(W.fault + blockIdx.x, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            // every wave's guard stores drained above: the record is whole
            uint32_t g[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                g[k] = __hip_atomic_load(W.brec + 4u * blockIdx.x + k, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
            if (g[0]) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    __hip_atomic_store(W.srec + 4u * si + k, g[k], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __hip_atomic_store(W.done + si,
                               t | (f ? kWorkerFault : 0ull) | (g[0] ? kWorkerGuard : 0ull),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        t_last = wall_clock64();
        t += gridDim.x;
    }
    if (threadIdx.x == 0) {
        __hip_atomic_store(W.next + blockIdx.x, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        // tells the host to retire this launch (stop the rest) and relaunch
        __hip_atomic_fetch_add(&W.wctl->exited, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------------------
// Synthetic traffic straight into HBM (bench / parity input), one thread per
// packet.  Bit-identical to oracle_synth() on the host.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void yrss_synth(yrss_synth_params p, uint64_t first,
                                                  uint32_t n, uint8_t *win,
                                                  uint32_t stride, uint16_t *len)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    uint32_t w[20];
    uint16_t L;
    yrss_synth_window(&p, first + i, w, &L);
    uint8_t *dst = win + (size_t)i * stride;
#pragma unroll
    for (int c = 0; c < 5; ++c)
        if ((uint32_t)c * 16u < stride)
            *reinterpret_cast<uint4 *>(dst + c * 16) =
                make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
    for (uint32_t c = 5; c * 16u < stride; ++c) {
        uint32_t v[4];
        for (int d = 0; d < 4; ++d) {
            uint32_t x = 0;
            for (int b = 0; b < 4; ++b) {
                const uint32_t k = c * 16u + d * 4u + b;
                x |= ((k * 131u + i) & 0xffu) << (8 * b);
            }
            v[d] = x;
        }
        *reinterpret_cast<uint4 *>(dst + c * 16) = make_uint4(v[0], v[1], v[2], v[3]);
    }
    len[i] = L;
}

}  // namespace

// ===========================================================================
// Host side
// ===========================================================================

struct TimedPair {
    hipEvent_t a, b;
    int kernel;
};

// A host output array: written in place when it is registered (the kernel or
// the DMA writes it directly), else through the context's pinned staging and
// copied when the burst completes.
struct HostOut {
    void *user;
    void *stage;
    size_t bytes;
    bool direct;
};

// The host-resident burst in flight on the context stream.  Synchronous calls
// complete it before returning; YRSS_F_ASYNC leaves it for yrss_wait.
struct PendingBurst {
    bool active = false;
    uint32_t n = 0;
    HostOut outs[5] = {};            // q, hash, qidx, qstart, filter
    bool gather_fault = false;       // zero-copy: a pointer outside every range
    bool dev_fault = false;          // multi-kernel path: check the fault record
    uint64_t done_seq = 0;           // one-launch path: value the kernel stores in *h_done
    void *const *wb_mbufs = nullptr; // host-side hash.rss write-back (staged path)
};

struct yrss_ctx {
    yrss_config cfg;
    int device = 0;
    int cus = 0;
    // Parse-kernel launch shape: one 512-thread workgroup (8 waves) per CU,
    // the best of the on-hardware sweeps (profiles/r01_sweep_*.json,
    // r01_v30_occupancy_ab.log: 12 resident waves were equal, 16 worse).
    // yrss_set_tuning overrides the layout for tests and measurements.
    yrss_tuning tune{};
    uint32_t nb = 0;
    ParseParams proto{};         // key schedule, modulo constants
    // KNI (protocol_filter) state, ff_dpdk_kni.c:60-61 / ff_dpdk_if.c:103-104
    bool kni_enable = false;
    bool kni_accept = false;
    uint8_t kni_bm[2 * 8192] = {};   // tcp bitmap then udp bitmap, htons-indexed
    uint32_t *d_kni = nullptr;
    struct Occ {
        const void *fn;
        uint32_t block, lds, blocks;
    };
    std::vector<Occ> occ;           // resident_blocks cache
    // The lists' workspace: per-chunk counts and prefixes, totals, scan
    // status, ranks.
    struct ListWs {
        uint32_t *seg_cnt = nullptr;
        uint32_t *seg_off = nullptr;
        uint32_t *totals = nullptr;
        unsigned long long *scan_status = nullptr;   // [nb][kMaxChunks / kScanTile]
        uint32_t scan_epoch = 0;
        uint16_t *rank = nullptr;    // n x u16, grown on demand
        size_t rank_cap = 0;
        // in-scatter prefixes: two sets of totals and range bins (the parse
        // kernel adds to set tot_set, its line scatter zeroes the other for
        // the next batch)
        uint32_t *tot_acc = nullptr;            // [2][nb]
        uint32_t tot_set = 0;
        uint32_t *rbin = nullptr;               // [2][kLbMaxWgs][nb]
    };
    ListWs ws;
    uint32_t *d_fault_rec = nullptr;    // host-coherent fault record {code, kernel, where, value}
    // host-burst staging (pinned) and its device mirror
    hipStream_t stream = nullptr;
    uint32_t burst_cap = 0;
    uint8_t *h_win = nullptr;
    uint16_t *h_len = nullptr;
    int16_t *h_q = nullptr;
    uint32_t *h_hash = nullptr;
    uint32_t *h_qidx = nullptr;
    uint32_t *h_qstart = nullptr;
    int8_t *h_filter = nullptr;
    uint8_t *d_win = nullptr;
    uint16_t *d_len = nullptr;
    int16_t *d_q = nullptr;
    uint32_t *d_hash = nullptr;
    uint32_t *d_qidx = nullptr;
    uint32_t *d_qstart = nullptr;
    int8_t *d_filter = nullptr;
    // zero-copy: registered host ranges, device pointer array and fault word
    uint32_t nranges = 0;
    HostRange ranges[YRSS_MAX_HOST_RANGES] = {};
    void *range_base[YRSS_MAX_HOST_RANGES] = {};
    uint64_t *h_ptrs = nullptr;
    uint64_t *d_ptrs = nullptr;
    uint32_t *d_fault = nullptr;
    uint32_t *h_fault = nullptr;    // host-coherent
    uint64_t *h_done = nullptr;     // host-coherent completion word of yrss_burst_small
    uint64_t *dh_done = nullptr;
    uint64_t done_seq = 0;
    // device views of the pinned staging: the small-burst kernel reads and
    // writes it in place (no copies)
    uint8_t *dh_win = nullptr;
    uint16_t *dh_len = nullptr;
    int16_t *dh_q = nullptr;
    uint32_t *dh_hash = nullptr;
    uint32_t *dh_qidx = nullptr;
    uint32_t *dh_qstart = nullptr;
    int8_t *dh_filter = nullptr;
    uint64_t *dh_ptrs = nullptr;
    uint32_t *dh_fault = nullptr;
    PendingBurst pend;
    // persistent burst worker (yrss_worker_*)
    struct WorkerState {
        bool on = false;           // yrss_worker_start called
        bool running = false;      // a worker launch may still be in flight
        uint32_t nslots = 0, nblocks = 0, qs_stride = 0;
        uint64_t idle_ticks = 0, life_ticks = 0;
        uint32_t poll_sleep = 1;
        hipStream_t stream = nullptr;
        WorkerSlot *slots = nullptr, *d_slots = nullptr;   // host-coherent
        uint64_t *done = nullptr, *d_done = nullptr;       // host-coherent
        uint32_t *fault = nullptr;                         // device [nblocks]
        uint32_t *brec = nullptr;                          // device [nblocks][4]
        uint32_t *srec = nullptr, *d_srec = nullptr;       // host-coherent [nslots][4]
        uint64_t *ptrs = nullptr, *d_ptrs = nullptr;       // pinned
        uint16_t *lens = nullptr, *d_lens = nullptr;       // pinned (frames mode)
        int16_t *q = nullptr, *d_q = nullptr;
        uint32_t *hash = nullptr, *d_hash = nullptr;
        uint32_t *qidx = nullptr, *d_qidx = nullptr;
        uint32_t *qstart = nullptr, *d_qstart = nullptr;
        uint64_t *next = nullptr, *d_next = nullptr;       // host-coherent
        WorkerCtl *ctl = nullptr, *d_ctl = nullptr;        // host-coherent
        uint8_t *win = nullptr;                            // device scratch
        uint16_t *len = nullptr;
        uint64_t issued = 0;       // last ticket handed out
        uint32_t pending = 0;      // submitted, not yet polled
        uint64_t *last_out = nullptr;   // [nslots][4] output addresses of each slot's last burst
        struct Out {
            int16_t *q;
            uint32_t *hash, *qidx, *qstart;
            uint32_t n;
            bool collected;
            uint8_t copy;          // bit k: output k comes from the slot's staging
        } *out = nullptr;          // [nslots]
    } w;
    // yrss_toeplitz_dispatch through the worker: one registered window slot
    uint8_t *shim_win = nullptr;
    // The compaction workspace is shared by every dispatch of the context; a
    // dispatch on a different stream than the previous one first waits for
    // the work queued on that stream (recorded at the switch, so same-stream
    // dispatches pay nothing).
    hipStream_t last_stream = nullptr;
    bool last_stream_valid = false;
    hipEvent_t switch_ev = nullptr;
    // timing
    uint32_t timing_mask = 0;    // bit k: bracket kernel k with events
    std::vector<hipEvent_t> ev_free;
    std::vector<TimedPair> ev_pending;
    double ms[YRSS_K_COUNT] = {0, 0, 0};
    uint32_t launches[YRSS_K_COUNT] = {0, 0, 0};
    std::vector<float> durs[YRSS_K_COUNT];   // per-launch ms since yrss_timing_enable
    // A call on this context saw the GPU not finish its work (-ETIMEDOUT):
    // yrss_fini then neither waits for the device nor frees memory a running
    // kernel may still touch (the allocations are left to process exit).
    bool hung = false;
    // Test hooks (set only through the yrss_debug_* entry points of a
    // -DYRSS_TEST_HOOKS build, libyrss_test.so; always 0 in libyrss.so).
    struct Debug {
        uint64_t worker_inject = 0;   // ticket whose worker burst fires a list guard
        uint32_t line_groups = 0;     // force the line scatter's kG (2 or 4)
        uint32_t skip_line_check = 0; // launch a line scatter the host check refuses
        uint32_t partial_merge = 0;   // partial list lines as plain stores
    } dbg;
};

namespace {

int hip_fail(const char *what, hipError_t e)
{
    fprintf(stderr, "yrss: %s failed: %s\n", what, hipGetErrorString(e));
    return -EIO;
}

#define YRSS_HIP(call)                                   \
    do {                                                 \
        hipError_t e_ = (call);                          \
        if (e_ != hipSuccess)                            \
            return hip_fail(#call, e_);                  \
    } while (0)

constexpr uint32_t kParseBlock = 512;   // 8 waves: one workgroup per CU (LDS)

size_t parse_lds(bool filter)
{
    constexpr size_t w = kParseBlock / kWave;
    return kTblBytes + w * kStageBytes + w * (kCntWords * sizeof(uint32_t) + kOutBytes) +
           (filter ? kKniWords * sizeof(uint32_t) : 0u);
}

// One workgroup per CU (the LDS of the filter variant admits no second), so
// the grid does not depend on whether the filter is on and a batch's layout
// (and its compaction) is the same for every variant.
uint32_t grid_for(const yrss_ctx *c, uint32_t n)
{
    const uint64_t per_block = (uint64_t)(kParseBlock / kWave) * kTile;
    const uint32_t want = (uint32_t)(((uint64_t)n + per_block - 1) / per_block);
    const uint32_t cap = c->tune.parse_blocks ? c->tune.parse_blocks : (uint32_t)c->cus;
    return std::max(1u, std::min(want, cap));
}

// Work layout of one launch.
// - chunk (2^ct_shift tiles): the unit the parse kernel deals round-robin to
//   its waves and counts per bucket.  Small chunks keep the chip's reads in a
//   compact window; each wave keeps one LDS count slot (nb words) per chunk it
//   owns, so chunks <= waves x (kCntWords / nb): 4 tiles up to 64 buckets at
//   2^24 packets, larger past that or past 2^24 packets.
// - span (2^shift chunks, 32 tiles = 2048 packets by default): one scatter
//   wave's unit, worked in pieces of kPiece packets.
// - ncol: chunk columns rounded up to whole scan tiles.
struct Layout {
    uint32_t chunk, ct_shift, shift, seg, nchunk, ncol;
};

Layout layout_for(const yrss_ctx *c, uint32_t n, uint32_t grid)
{
    const uint64_t waves = (uint64_t)grid * (kParseBlock / kWave);
    const uint64_t slots = std::max<uint32_t>(1u, kCntWords / c->nb);
    const uint64_t max_chunks = std::min<uint64_t>(kMaxChunks, waves * slots);
    const uint64_t tiles = ((uint64_t)n + kTile - 1) / kTile;
    // Fewer, larger chunks mean fewer per-chunk counts for the parse kernel
    // to flush and the scan to pass over, but a coarser deal of the batch to
    // the parse waves: 4 tiles up to 16 buckets (8 tiles cost the parse ~7 us
    // at 9 buckets), 8 tiles to 128 (the scan 9.8 -> 6.4 us at 65 buckets,
    // r03 A/B; the bucket still packs beside a 9-bit rank).  Past 128 buckets
    // the rank sits beside q whatever the chunk, and two chunks a wave, up to
    // 64 tiles, were fastest (256 buckets at 2^24 packets, 16 -> 32 -> 64
    // tiles: step 0.3046 -> 0.3012 -> 0.2961 ms, scan 8.2 -> 5.0 -> 4.7 us,
    // scatter 64 -> 62 -> 60 us; 128 tiles no better;
    // profiles/r04_chunk32_grouped_ab.log, r04_chunk_sweep_{a,b}.log)
    uint64_t ct_many = 16u;
    while (ct_many < 64u && ct_many * 2u * 2u * waves <= tiles)
        ct_many *= 2u;
    const uint64_t ct_nb = c->nb <= 16u ? 4u : c->nb <= 128u ? 8u : ct_many;
    uint64_t ct = std::max<uint64_t>(c->tune.chunk_tiles ? c->tune.chunk_tiles : ct_nb,
                                     (tiles + max_chunks - 1) / max_chunks);
    uint32_t ct_shift = 0;
    while ((1ull << ct_shift) < ct)
        ++ct_shift;
    ct = 1ull << ct_shift;
    const uint64_t st = c->tune.span_tiles ? c->tune.span_tiles : kPiece / kTile;
    Layout L;
    L.ct_shift = ct_shift;
    L.shift = 0;
    while ((ct << L.shift) < st)
        ++L.shift;
    L.chunk = (uint32_t)(ct * kTile);
    L.seg = L.chunk << L.shift;
    L.nchunk = (uint32_t)(((uint64_t)n + L.chunk - 1) / L.chunk);
    L.ncol = (L.nchunk + kScanTile - 1) / kScanTile * kScanTile;
    return L;
}

// LDS of one wave of the fallback scatter (yrss_scatter): six per-bucket
// arrays and the stage (a piece plus up to 3 words of alignment padding per
// bucket); wpb waves per workgroup, halved until a workgroup holds at most
// 64 KiB.
struct ScatterLds {
    uint32_t aux, stg, wlds, wpb;
};
constexpr uint32_t kScatterLdsMax = 64u * 1024u / 4u;   // words per workgroup

ScatterLds scatter_lds(uint32_t nb)
{
    ScatterLds r;
    r.stg = (kPiece + 3u * nb + 3u) & ~3u;
    r.aux = (6u * nb + 3u) & ~3u;
    r.wlds = r.aux + r.stg;
    r.wpb = (uint32_t)kScatterWaves;
    while (r.wpb > 1 && r.wpb * r.wlds > kScatterLdsMax)
        r.wpb /= 2;
    return r;
}

// The line scatter's span and stage for a layout: spans of up to
// kLineSpanMax packets (yrss_tuning.span_tiles lowers it), as many chunks as
// keep the prefix table within line_tab_max words; none when a chunk is longer
// than a span can be (batches past ~2^29 packets) or the LDS would not fit.
struct LinePlan {
    bool ok, packed;
    bool fits;   // nb within the kernel's per-bucket capacity (line_nb_max)
    uint32_t groups, gshift, seg, lmax, lds;
};

LinePlan line_plan(const yrss_ctx *c, const Layout &lay)
{
    LinePlan p{};
    const uint32_t nb = c->nb, cshift = lay.ct_shift + 6u;
    // kG = 2 up to 128 buckets, 4 past that (the test hook forces one)
    p.groups = c->dbg.line_groups ? c->dbg.line_groups : nb > line_nb_max(2) ? 4u : 2u;
    p.fits = nb <= line_nb_max(p.groups) && nb <= (uint32_t)kLineBlock;
    const uint32_t smax = line_span_max(p.groups);
    const uint32_t tmax = line_tab_max(p.groups);
    if (lay.chunk > smax || nb > (uint32_t)kLineBlock)
        return p;
    uint64_t target = c->tune.span_tiles ? (uint64_t)c->tune.span_tiles * kTile : smax;
    target = std::min<uint64_t>(std::max<uint64_t>(target, lay.chunk), smax);
    p.gshift = 0;
    while (((uint64_t)lay.chunk << (p.gshift + 1)) <= target &&
           ((uint64_t)nb << (p.gshift + 1)) <= tmax)
        ++p.gshift;
    if (((uint64_t)nb << p.gshift) > tmax)
        return p;
    p.seg = lay.chunk << p.gshift;
    p.lmax = p.seg / 16u + 2u * nb + 1u;   // a bucket's lines <= (its packets + 30) / 16
    // the tagging's lines a thread (kTagLines) must reach every stage line
    p.fits = p.fits && p.lmax <= (uint32_t)kLineBlock * (p.groups == 4u ? 5u : 2u);
    p.lds = line_lds(nb, p.gshift, p.lmax).words * 4u;
    if (p.lds > 160u * 1024u)
        return p;
    // bucket << cshift | rank fits 16 bits
    p.packed = cshift < 16u && nb <= (1u << (16u - cshift));
    p.ok = true;
    return p;
}

// Workgroups of kernel fn (block threads, lds bytes) resident on the whole
// device at once, from the occupancy calculator, cached per context.
uint32_t resident_blocks(yrss_ctx *c, const void *fn, uint32_t block, uint32_t lds)
{
    for (const auto &e : c->occ)
        if (e.fn == fn && e.block == block && e.lds == lds)
            return e.blocks;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, (int)block, lds) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    const uint32_t blocks = (uint32_t)per_cu * (uint32_t)c->cus;
    c->occ.push_back({fn, block, lds, blocks});
    return blocks;
}

typedef void (*ParseKernel)(ParseParams);

// count: 0 none, 1 per-chunk counts, 2 counts + per-packet chunk ranks
ParseKernel pick_parse(int count, bool filter)
{
    if (filter)
        return count == 2 ? yrss_parse_hash<2, true, kParseBlock>
               : count    ? yrss_parse_hash<1, true, kParseBlock>
                          : yrss_parse_hash<0, true, kParseBlock>;
    return count == 2 ? yrss_parse_hash<2, false, kParseBlock>
           : count    ? yrss_parse_hash<1, false, kParseBlock>
                      : yrss_parse_hash<0, false, kParseBlock>;
}

hipEvent_t take_event(yrss_ctx *c)
{
    if (c->ev_free.empty()) {
        // Device-scope release: the outputs are consumed by later kernels on
        // this device, and the host synchronises on the stream anyway.  The
        // default system-scope fence writes back L2 at each timed kernel's end.
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess)
            return nullptr;
        return e;
    }
    hipEvent_t e = c->ev_free.back();
    c->ev_free.pop_back();
    return e;
}

// Per-kernel timing: the events ride on the kernel's own AQL dispatch packet
// (hipExtLaunchKernel), so timing adds no marker packets to the stream, and
// they are created with hipEventDisableSystemFence (device-scope release).
// hipEventRecord markers with the default system-scope fence left ~6 us of
// idle GPU before and after the timed kernel (profiles/r01_v8_*), ~5 % of a
// step; with both changes the bench step is within ~1 us of an untimed one.
struct Timed {
    yrss_ctx *c;
    int k;
    hipEvent_t a = nullptr, b = nullptr;
    Timed(yrss_ctx *c_, int k_) : c(c_), k(k_)
    {
        if ((c->timing_mask >> k) & 1u) {
            a = take_event(c);
            b = take_event(c);
            if (!a || !b)
                a = b = nullptr;
        }
    }
    ~Timed()
    {
        if (a && b)
            c->ev_pending.push_back({a, b, k});
    }
};

void compute_key_schedule(const yrss_config *cfg, uint32_t kwin[96])
{
    for (unsigned k = 0; k < 96; ++k) {
        uint32_t w = 0;
        for (unsigned b = 0; b < 32; ++b) {
            const unsigned bit = k + b, kb = bit >> 3;
            const unsigned v =
                kb < cfg->rss_key_len ? (cfg->rss_key[kb] >> (7 - (bit & 7))) & 1u : 0u;
            w = (w << 1) | v;
        }
        kwin[k] = w;
    }
}

// set_bitmap (ff_dpdk_kni.c:84-89): bit 0x80 >> (p % 8) of byte p / 8, p = htons(port)
void kni_set_port(uint8_t *bm, uint16_t port)
{
    const uint16_t p = (uint16_t)((port << 8) | (port >> 8));
    bm[p >> 3] |= (uint8_t)(0x80u >> (p & 7u));
}

// kni_set_bitmap (ff_dpdk_kni.c:99-118), same tokenising rules: a '-' before
// the next ',' (with at least one character between) makes a range, both ends
// via atoi; every value goes through the uint16_t of set_bitmap.
void kni_parse_ports(const char *p, uint8_t *bm)
{
    if (!p)
        return;
    const char *head = p;
    for (;;) {
        const char *tail = strstr(head, ",");
        const char *tail_num = strstr(head, "-");
        if (tail_num && (!tail || tail_num < tail - 1)) {
            const long lo = atoi(head), hi = atoi(tail_num + 1);
            // a range of 65536+ values sets every bit; bound the loop there
            for (long i = lo, k = 0; i <= hi && k < 65536; ++i, ++k)
                kni_set_port(bm, (uint16_t)i);
        } else {
            kni_set_port(bm, (uint16_t)atoi(head));
        }
        if (!tail)
            break;
        head = tail + 1;
    }
}

void free_burst(yrss_ctx *c)
{
    (void)hipHostFree(c->h_win); (void)hipHostFree(c->h_len); (void)hipHostFree(c->h_q);
    (void)hipHostFree(c->h_hash); (void)hipHostFree(c->h_qidx); (void)hipHostFree(c->h_qstart);
    (void)hipHostFree(c->h_filter);
    (void)hipHostFree(c->h_ptrs);
    (void)hipFree(c->d_ptrs);
    c->h_ptrs = nullptr;
    c->d_ptrs = nullptr;
    (void)hipFree(c->d_win); (void)hipFree(c->d_len); (void)hipFree(c->d_q);
    (void)hipFree(c->d_hash); (void)hipFree(c->d_qidx); (void)hipFree(c->d_qstart);
    (void)hipFree(c->d_filter);
    c->h_win = nullptr; c->h_len = nullptr; c->h_q = nullptr; c->h_hash = nullptr;
    c->h_qidx = nullptr; c->h_qstart = nullptr; c->h_filter = nullptr;
    c->d_win = nullptr; c->d_len = nullptr; c->d_q = nullptr; c->d_hash = nullptr;
    c->d_qidx = nullptr; c->d_qstart = nullptr; c->d_filter = nullptr;
    c->burst_cap = 0;
}

int ensure_burst(yrss_ctx *c, uint32_t n)
{
    if (n <= c->burst_cap)
        return 0;
    free_burst(c);
    const uint32_t cap = std::max<uint32_t>(n, 1024u);
    const size_t nbk = (size_t)c->nb + 1;
    YRSS_HIP(hipHostMalloc((void **)&c->h_win, (size_t)cap * YRSS_WIN_FULL, hipHostMallocDefault));
    YRSS_HIP(hipHostMalloc((void **)&c->h_len, (size_t)cap * 2, hipHostMallocDefault));
    YRSS_HIP(hipHostMalloc((void **)&c->h_q, (size_t)cap * 2, hipHostMallocDefault));
    YRSS_HIP(hipHostMalloc((void **)&c->h_hash, (size_t)cap * 4, hipHostMallocDefault));
    YRSS_HIP(hipHostMalloc((void **)&c->h_qidx, (size_t)cap * 4, hipHostMallocDefault));
    YRSS_HIP(hipHostMalloc((void **)&c->h_qstart, nbk * 4, hipHostMallocDefault));
    YRSS_HIP(hipHostMalloc((void **)&c->h_filter, (size_t)cap, hipHostMallocDefault));
    YRSS_HIP(hipMalloc((void **)&c->d_win, (size_t)cap * YRSS_WIN_FULL));
    YRSS_HIP(hipMalloc((void **)&c->d_len, (size_t)cap * 2));
    YRSS_HIP(hipMalloc((void **)&c->d_q, (size_t)cap * 2));
    YRSS_HIP(hipMalloc((void **)&c->d_hash, (size_t)cap * 4));
    YRSS_HIP(hipMalloc((void **)&c->d_qidx, (size_t)cap * 4));
    YRSS_HIP(hipMalloc((void **)&c->d_qstart, nbk * 4));
    YRSS_HIP(hipMalloc((void **)&c->d_filter, (size_t)cap));
    YRSS_HIP(hipHostMalloc((void **)&c->h_ptrs, (size_t)cap * 8, hipHostMallocDefault));
    YRSS_HIP(hipMalloc((void **)&c->d_ptrs, (size_t)cap * 8));
    YRSS_HIP(hipHostGetDevicePointer((void **)&c->dh_win, c->h_win, 0));
    YRSS_HIP(hipHostGetDevicePointer((void **)&c->dh_len, c->h_len, 0));
    YRSS_HIP(hipHostGetDevicePointer((void **)&c->dh_q, c->h_q, 0));
    YRSS_HIP(hipHostGetDevicePointer((void **)&c->dh_hash, c->h_hash, 0));
    YRSS_HIP(hipHostGetDevicePointer((void **)&c->dh_qidx, c->h_qidx, 0));
    YRSS_HIP(hipHostGetDevicePointer((void **)&c->dh_qstart, c->h_qstart, 0));
    YRSS_HIP(hipHostGetDevicePointer((void **)&c->dh_filter, c->h_filter, 0));
    YRSS_HIP(hipHostGetDevicePointer((void **)&c->dh_ptrs, c->h_ptrs, 0));
    c->burst_cap = cap;
    return 0;
}

// Host-staged classification shared by the burst/frames/route entry points.
// The windows and data_len are already gathered into c->h_win / c->h_len at
// stride W; results land in the caller's host arrays (NULL = not wanted).
// hipHostRegister is process-wide, but each context keeps its own range table
// (several contexts pipeline bursts over one mbuf pool), so registrations are
// reference-counted per (base, len).
// A range of a context closed after a GPU timeout is poisoned, not released:
// a kernel that never finished may still read or write it, so it stays
// registered for the life of the process, and registering that base again
// fails (the application must not reuse the pool's address for a new one).
struct HostReg {
    size_t len;
    uint32_t refs;
    bool poisoned;
};
std::mutex g_reg_mu;
std::map<void *, HostReg> g_reg;

hipError_t host_reg_acquire(void *base, size_t len)
{
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.find(base);
    if (it != g_reg.end()) {
        if (it->second.len != len || it->second.poisoned)
            return hipErrorHostMemoryAlreadyRegistered;
        ++it->second.refs;
        return hipSuccess;
    }
    const hipError_t e = hipHostRegister(base, len, hipHostRegisterMapped);
    if (e == hipSuccess)
        g_reg[base] = HostReg{len, 1u, false};
    return e;
}

void host_reg_release(void *base)
{
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.find(base);
    if (it == g_reg.end() || it->second.refs == 0)
        return;
    if (--it->second.refs == 0 && !it->second.poisoned) {
        (void)hipHostUnregister(base);
        g_reg.erase(it);
    }
}

// the hung-context path of yrss_fini: the context's reference is dropped,
// the range stays registered and refuses new registrations
void host_reg_poison(void *base)
{
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.find(base);
    if (it == g_reg.end())
        return;
    it->second.poisoned = true;
    if (it->second.refs)
        --it->second.refs;
}

int worker_halt(yrss_ctx *c);
void worker_free(yrss_ctx *c);

uint64_t mono_ns()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// Context behind yrss_toeplitz_dispatch: dispatch_func_t has no context
// argument (ff_api.h:167), so the registration shim reads this one.  The
// mutex serialises shim calls: with soft_dispatch=0 every lcore calls the
// registered dispatcher (ff_dpdk_if.c:1653,1078), and one context's staging
// and burst state take one burst at a time.  yrss_fini takes it too, so a
// context is never torn down under a running shim call.
yrss_ctx *g_dispatch_ctx = nullptr;
std::mutex g_dispatch_mu;

const char *fault_name(uint32_t code)
{
    switch (code) {
    case YRSS_FAULT_SCAN_TIMEOUT: return "scan look-back did not resolve";
    case YRSS_FAULT_LIST_RANGE: return "list slot outside the batch";
    case YRSS_FAULT_COUNT_MISMATCH: return "span histogram differs from the parse counts";
    case YRSS_FAULT_COUNT_SLOT: return "parse count slot outside the wave's LDS";
    case YRSS_FAULT_STAGE: return "stage slot outside the piece";
    case YRSS_FAULT_LINE_CAPACITY: return "line scatter launched for more buckets than it holds";
    default: return "unknown";
    }
}

// A device-side guard that fired (the fault record is set) leaves that
// batch's per-queue lists invalid; q and hash are not affected.  Copies the
// record to *out (if given) and clears it.  The caller has synchronised.
bool take_fault(yrss_ctx *c, yrss_fault *out = nullptr)
{
    uint32_t *r = c->d_fault_rec;
    const yrss_fault f{__atomic_load_n(r, __ATOMIC_ACQUIRE), r[1], r[2], r[3]};
    if (out)
        *out = f;
    if (!f.code)
        return false;
    fprintf(stderr, "yrss: device fault %u (%s) in %s at %u (value %u); per-queue lists invalid\n",
            f.code, fault_name(f.code), yrss_kernel_name((int)f.kernel), f.where, f.value);
    r[1] = r[2] = r[3] = 0u;
    __atomic_store_n(r, 0u, __ATOMIC_RELEASE);
    return true;
}

int dispatch_dev_impl(yrss_ctx *c, const struct yrss_dev_batch *b, void *stream);

// The lists' workspace (the count matrix zeroed: the parse kernel writes only
// the columns of the launch)
hipError_t list_ws_alloc(yrss_ctx *c, yrss_ctx::ListWs &w)
{
    const size_t cnt = (size_t)kMaxChunks * c->nb * sizeof(uint32_t);
    const size_t st = (size_t)c->nb * (kMaxChunks / kScanTile) * sizeof(unsigned long long);
    hipError_t e;
    if ((e = hipMalloc((void **)&w.seg_cnt, cnt)) != hipSuccess ||
        (e = hipMalloc((void **)&w.seg_off, cnt)) != hipSuccess ||
        (e = hipMalloc((void **)&w.totals, c->nb * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc((void **)&w.scan_status, st)) != hipSuccess ||
        (e = hipMemset(w.scan_status, 0, st)) != hipSuccess ||
        (e = hipMemset(w.seg_cnt, 0, cnt)) != hipSuccess)
        return e;
    if (c->nb <= kFusedMaxNb) {
        const size_t rb = 2u * kLbMaxWgs * c->nb * sizeof(uint32_t);
        if ((e = hipMalloc((void **)&w.tot_acc, 2u * c->nb * sizeof(uint32_t))) != hipSuccess ||
            (e = hipMemset(w.tot_acc, 0, 2u * c->nb * sizeof(uint32_t))) != hipSuccess ||
            (e = hipMalloc((void **)&w.rbin, rb)) != hipSuccess ||
            (e = hipMemset(w.rbin, 0, rb)) != hipSuccess)
            return e;
    }
    return hipSuccess;
}

void list_ws_free(yrss_ctx::ListWs &w)
{
    (void)hipFree(w.seg_cnt);
    (void)hipFree(w.seg_off);
    (void)hipFree(w.totals);
    (void)hipFree(w.scan_status);
    (void)hipFree(w.tot_acc);
    (void)hipFree(w.rbin);
    (void)hipFree(w.rank);
    w = yrss_ctx::ListWs{};
}

bool small_ok(const yrss_ctx *c, uint32_t n)
{
    return c->tune.one_launch != 2 && n >= 1 && n <= kSmallMaxPkts && c->nb <= kSmallMaxNb;
}

// One launch of yrss_burst_small on the context stream.  S.P.win/len and the
// output pointers are filled by the caller; this adds the configuration.
// host_burst: a host-resident burst on the context stream, completed by the
// host spinning on the kernel's completion word; otherwise a device batch on
// the caller's stream (no completion word).
int small_launch(yrss_ctx *c, SmallParams &S, bool filter, bool host_burst = true,
                 hipStream_t stream = nullptr)
{
    const ParseParams &proto = c->proto;
    ParseParams &P = S.P;
    memcpy(P.kwin, proto.kwin, sizeof(P.kwin));
    P.nq = proto.nq;
    P.nb = proto.nb;
    P.mod_d = proto.mod_d;
    P.q_off = proto.q_off;
    P.mod_m = proto.mod_m;
    P.seg_cnt = nullptr;
    P.rank = nullptr;
    P.fault = c->d_fault_rec;
    P.kni_bm = c->d_kni;
    P.kni_enable = c->kni_enable ? 1u : 0u;
    if (host_burst) {
        S.done = c->dh_done;
        S.seq = ++c->done_seq;
        c->pend.done_seq = S.seq;   // the caller reset pend before
        stream = c->stream;
    } else {
        S.done = nullptr;
    }
    const size_t lds = small_lds(c->nb, filter);
    const dim3 grid(1);
    if (filter)
        hipLaunchKernelGGL(yrss_burst_small<true>, grid, dim3(kSmallBlock), lds, stream, S);
    else
        hipLaunchKernelGGL(yrss_burst_small<false>, grid, dim3(kSmallBlock), lds, stream, S);
    YRSS_HIP(hipGetLastError());
    return 0;
}

// Completes the pending host burst: waits for the stream, checks the device
// fault words, copies staged outputs and writes hash.rss back on the host.
int finish_burst(yrss_ctx *c)
{
    PendingBurst &p = c->pend;
    if (!p.active)
        return 0;
    p.active = false;
    // One-launch bursts publish a completion word: spin on it (a stream
    // synchronisation costs microseconds of wake-up on top of the kernel);
    // anything else, or a word that does not come, takes the stream sync.
    bool done = false;
    if (p.done_seq) {
        const uint64_t t0 = mono_ns();
        for (uint32_t k = 1;; ++k) {
            if (__atomic_load_n(c->h_done, __ATOMIC_ACQUIRE) == p.done_seq) {
                done = true;
                break;
            }
            if ((k & 255u) == 0 && mono_ns() - t0 > 2000000ull)   // 2 ms
                break;
            __builtin_ia32_pause();
        }
    }
    if (!done)
        YRSS_HIP(hipStreamSynchronize(c->stream));
    if (p.gather_fault && __atomic_load_n(c->h_fault, __ATOMIC_ACQUIRE))
        return -EFAULT;
    if (p.dev_fault && take_fault(c))
        return -EIO;
    for (int k = 0; k < 5; ++k)
        if (p.outs[k].user && !p.outs[k].direct)
            memcpy(p.outs[k].user, p.outs[k].stage, p.outs[k].bytes);
    if (p.wb_mbufs) {
        const uint8_t *h = (const uint8_t *)(p.outs[1].user ? p.outs[1].user : p.outs[1].stage);
        for (uint32_t i = 0; i < p.n; ++i)
            memcpy((uint8_t *)p.wb_mbufs[i] + c->cfg.mbuf.off_hash_rss, h + 4u * i, 4);
    }
    return 0;
}

// Queues the classification of windows already gathered into c->h_win /
// c->h_len at stride W; results go to the caller's host arrays (NULL = not
// wanted) when the burst completes (finish_burst).  want_hash computes the
// hash into the staging even without out_hash (hash.rss write-back).
int classify_staged(yrss_ctx *c, uint32_t n, uint32_t W, int16_t *out_q, uint32_t *out_hash,
                    uint32_t *out_qidx, uint32_t *out_qstart, int8_t *out_filter, bool want_hash)
{
    hipStream_t s = c->stream;
    const bool compact = out_qidx && out_qstart;
    want_hash = want_hash || out_hash;
    PendingBurst &p = c->pend;
    p = PendingBurst{};
    p.n = n;
    p.outs[0] = {out_q, c->h_q, (size_t)n * 2, false};
    p.outs[1] = {out_hash, c->h_hash, (size_t)n * 4, false};
    p.outs[2] = {compact ? out_qidx : nullptr, c->h_qidx, (size_t)n * 4, false};
    p.outs[3] = {compact ? out_qstart : nullptr, c->h_qstart, (c->nb + 1) * 4, false};
    p.outs[4] = {out_filter, c->h_filter, n, false};
    if (small_ok(c, n)) {
        // the kernel reads the staged windows and writes the staging in place
        SmallParams S;
        memset(&S, 0, sizeof(S));
        S.P.win = c->dh_win;
        S.P.len = c->dh_len;
        S.P.stride = W;
        S.P.n = n;
        S.P.q = c->dh_q;
        S.P.hash = want_hash ? c->dh_hash : nullptr;
        S.P.filter = out_filter ? c->dh_filter : nullptr;
        S.qidx = compact ? c->dh_qidx : nullptr;
        S.qstart = compact ? c->dh_qstart : nullptr;
        int rc = small_launch(c, S, out_filter != nullptr);
        if (rc)
            return rc;
        p.active = true;
        return 0;
    }
    YRSS_HIP(hipMemcpyAsync(c->d_win, c->h_win, (size_t)n * W, hipMemcpyHostToDevice, s));
    YRSS_HIP(hipMemcpyAsync(c->d_len, c->h_len, (size_t)n * 2, hipMemcpyHostToDevice, s));
    yrss_dev_batch b;
    b.win = c->d_win;
    b.win_stride = W;
    b.n = n;
    b.len = c->d_len;
    b.q = c->d_q;
    b.hash = want_hash ? c->d_hash : nullptr;
    b.qidx = compact ? c->d_qidx : nullptr;
    b.qstart = compact ? c->d_qstart : nullptr;
    b.filter = out_filter ? c->d_filter : nullptr;
    int rc = dispatch_dev_impl(c, &b, s);
    if (rc)
        return rc;
    YRSS_HIP(hipMemcpyAsync(c->h_q, c->d_q, (size_t)n * 2, hipMemcpyDeviceToHost, s));
    if (want_hash)
        YRSS_HIP(hipMemcpyAsync(c->h_hash, c->d_hash, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    if (out_filter)
        YRSS_HIP(hipMemcpyAsync(c->h_filter, c->d_filter, n, hipMemcpyDeviceToHost, s));
    if (compact) {
        YRSS_HIP(hipMemcpyAsync(c->h_qidx, c->d_qidx, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        YRSS_HIP(hipMemcpyAsync(c->h_qstart, c->d_qstart, (c->nb + 1) * 4,
                                hipMemcpyDeviceToHost, s));
    }
    p.dev_fault = compact;
    p.active = true;
    return 0;
}

// Host entry points: one burst in flight per context.  begin_burst refuses a
// second one; end_burst completes it unless the caller asked for YRSS_F_ASYNC.
int begin_burst(const yrss_ctx *c) { return c->pend.active ? -EBUSY : 0; }

int end_burst(yrss_ctx *c, uint32_t flags)
{
    return (flags & YRSS_F_ASYNC) ? 0 : finish_burst(c);
}

// Window stride for a host batch: 64 bytes when every frame fits, else 80
// (enough for any hash; KNI header walks past 80 bytes report TRUNC).
uint32_t host_stride(uint32_t maxlen) { return maxlen <= YRSS_WIN_MIN ? YRSS_WIN_MIN : YRSS_WIN_FULL; }

// Gather rte_mbuf first-segment headers (rte_pktmbuf_mtod, rte_mbuf.h:1620;
// rte_pktmbuf_data_len, ff_dpdk_if.c:1076) into the pinned staging.
int gather_mbufs(yrss_ctx *c, void *const *mbufs, uint32_t n, uint32_t *W_out)
{
    int rc = ensure_burst(c, n);
    if (rc)
        return rc;
    const yrss_mbuf_layout &ml = c->cfg.mbuf;
    // Two passes, both bound by host memory latency (cache-cold mbufs): the
    // first reads each header (data_len decides the window stride, and the
    // window's address is kept in the pinned pointer scratch), the second
    // copies the windows.  Each pass prefetches kGatherAhead packets ahead.
    constexpr uint32_t kGatherAhead = 16;
    const uint8_t **src = reinterpret_cast<const uint8_t **>(c->h_ptrs);
    uint32_t maxlen = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (i + kGatherAhead < n)
            __builtin_prefetch((const uint8_t *)mbufs[i + kGatherAhead]);
        const uint8_t *m = (const uint8_t *)mbufs[i];
        const uint8_t *buf;
        uint16_t doff, L;
        memcpy(&buf, m + ml.off_buf_addr, sizeof(buf));
        memcpy(&doff, m + ml.off_data_off, 2);
        memcpy(&L, m + ml.off_data_len, 2);
        src[i] = buf + doff;
        c->h_len[i] = L;
        maxlen = std::max<uint32_t>(maxlen, L);
    }
    const uint32_t W = host_stride(maxlen);
    for (uint32_t i = 0; i < n; ++i) {
        if (i + kGatherAhead < n) {
            __builtin_prefetch(src[i + kGatherAhead]);
            __builtin_prefetch(src[i + kGatherAhead] + W - 1);
        }
        const uint32_t L = c->h_len[i];
        memcpy(c->h_win + (size_t)i * W, src[i], L < W ? L : W);
    }
    *W_out = W;
    return 0;
}

}  // namespace

extern "C" {

const char *yrss_version(void) { return YRSS_VERSION_STRING; }

const char *yrss_kernel_name(int k)
{
    switch (k) {
    case YRSS_K_PARSE_HASH: return "yrss_parse_hash";
    case YRSS_K_SCAN: return "yrss_seg_scan";
    case YRSS_K_SCATTER: return "yrss_scatter";
    case YRSS_K_BURST: return "yrss_burst_small";
    case YRSS_K_WORKER: return "yrss_burst_worker";
    default: return "";
    }
}

void yrss_config_default(struct yrss_config *cfg)
{
    // Mellanox Linux driver key, ff_dpdk_if.c:113-119.
    static const uint8_t mlx_key[YRSS_RSS_KEY_LEN] = {
        0xd1, 0x81, 0xc6, 0x2c, 0xf7, 0xf4, 0xdb, 0x5b, 0x19, 0x83,
        0xa2, 0xfc, 0x94, 0x3e, 0x1a, 0xdb, 0xd9, 0x38, 0x9e, 0x6b,
        0xd1, 0x03, 0x9c, 0x2c, 0xa7, 0x44, 0x99, 0xad, 0x59, 0x3d,
        0x56, 0xd9, 0xf3, 0x25, 0x3c, 0x06, 0x2a, 0xdc, 0x1f, 0xfc};
    memset(cfg, 0, sizeof(*cfg));
    memcpy(cfg->rss_key, mlx_key, sizeof(mlx_key));
    cfg->rss_key_len = YRSS_RSS_KEY_LEN;
    cfg->nb_procs = 3;            // fs/config/config.ini lcore_mask=7
    cfg->nb_queues = 3;
    cfg->soft_dispatch = 1;       // config.ini soft_dispatch=1
    cfg->dispatch_only_core = 1;  // config.ini [system] dispatch_only_core=1
    cfg->device = 0;
    cfg->max_burst = 1u << 16;
    cfg->mbuf.off_buf_addr = YRSS_MBUF_OFF_BUF_ADDR;
    cfg->mbuf.off_data_off = YRSS_MBUF_OFF_DATA_OFF;
    cfg->mbuf.off_data_len = YRSS_MBUF_OFF_DATA_LEN;
    cfg->mbuf.off_hash_rss = YRSS_MBUF_OFF_HASH_RSS;
}

int yrss_config_validate(const struct yrss_config *cfg)
{
    if (!cfg)
        return -EINVAL;
    if (cfg->rss_key_len < 4 || cfg->rss_key_len > YRSS_RSS_KEY_LEN)
        return -EINVAL;
    if (cfg->nb_procs < 1 || cfg->nb_procs > YRSS_MAX_PROCS)
        return -EINVAL;
    if (cfg->nb_queues < 1 || cfg->nb_queues > YRSS_MAX_QUEUES)
        return -EINVAL;
    if (cfg->soft_dispatch > 1 || cfg->dispatch_only_core > 1)
        return -EINVAL;
    // hash % (nb_procs - 1) would divide by zero (ff_dpdk_if.c:2032)
    if (cfg->soft_dispatch && cfg->dispatch_only_core && cfg->nb_procs < 2)
        return -EINVAL;
    if (cfg->device < 0)
        return -EINVAL;
    return 0;
}

int yrss_init(const struct yrss_config *cfg, yrss_ctx **out)
{
    if (!out)
        return -EINVAL;
    *out = nullptr;
    int rc = yrss_config_validate(cfg);
    if (rc)
        return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= cfg->device)
        return -ENODEV;
    YRSS_HIP(hipSetDevice(cfg->device));
    hipDeviceProp_t prop;
    YRSS_HIP(hipGetDeviceProperties(&prop, cfg->device));

    yrss_ctx *c = new (std::nothrow) yrss_ctx();
    if (!c)
        return -ENOMEM;
    c->cfg = *cfg;
    c->device = cfg->device;
    c->cus = prop.multiProcessorCount;
    c->tune.scatter_xcd = -1;
    c->proto.out16 = 1;   // 16-byte write-through bursts (profiles/r01_v13_ahead_out16_ab.log)
    c->nb = (uint32_t)cfg->nb_queues + 1u;
    compute_key_schedule(cfg, c->proto.kwin);
    const bool only = cfg->soft_dispatch && cfg->dispatch_only_core;
    c->proto.mod_d = (uint32_t)(only ? cfg->nb_procs - 1 : cfg->nb_procs);
    c->proto.q_off = only ? 1u : 0u;
    c->proto.mod_m = UINT64_MAX / c->proto.mod_d + 1u;   // wraps to 0 for d == 1
    c->proto.nq = cfg->nb_queues;
    c->proto.nb = c->nb;

    const size_t ws = (size_t)kMaxChunks * c->nb * sizeof(uint32_t);
    hipError_t e;
    (void)ws;
    if ((e = list_ws_alloc(c, c->ws)) != hipSuccess ||
        (e = hipHostMalloc((void **)&c->d_fault_rec, 64, hipHostMallocCoherent)) != hipSuccess ||
        (e = hipMalloc((void **)&c->d_kni, sizeof(c->kni_bm))) != hipSuccess ||
        (e = hipMalloc((void **)&c->d_fault, sizeof(uint32_t))) != hipSuccess ||
        (e = hipHostMalloc((void **)&c->h_fault, sizeof(uint32_t), hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&c->dh_fault, c->h_fault, 0)) != hipSuccess ||
        (e = hipHostMalloc((void **)&c->h_done, 64, hipHostMallocCoherent)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&c->dh_done, c->h_done, 0)) != hipSuccess ||
        (e = hipMemset(c->d_kni, 0, sizeof(c->kni_bm))) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->switch_ev, hipEventDisableTiming)) != hipSuccess) {
        yrss_fini(c);
        return hip_fail("yrss_init allocation", e);
    }
    memset(c->d_fault_rec, 0, 64);
    *c->h_done = 0;
    // The memsets above run on the null stream, which does not order against
    // the context's non-blocking stream: without this wait a first dispatch
    // could race the zeroing of the count matrix (seen once on the GPU box as
    // short per-queue totals on a fresh context).
    if ((e = hipDeviceSynchronize()) != hipSuccess) {
        yrss_fini(c);
        return hip_fail("yrss_init synchronize", e);
    }
    if (cfg->max_burst && (rc = ensure_burst(c, cfg->max_burst)) != 0) {
        yrss_fini(c);
        return rc;
    }
    *out = c;
    return 0;
}

void yrss_fini(yrss_ctx *c)
{
    if (!c)
        return;
    (void)hipSetDevice(c->device);
    {
        std::lock_guard<std::mutex> lk(g_dispatch_mu);
        if (g_dispatch_ctx == c)
            g_dispatch_ctx = nullptr;
    }
    if (c->hung) {
        // A call already timed out on this device: draining it
        // would block here as well.  Ask a resident worker to leave, keep
        // every device and pinned allocation (a kernel still running may
        // write them), and free only what the host alone uses.
        if (c->w.on && c->w.ctl)
            __atomic_store_n(&c->w.ctl->stop, 1u, __ATOMIC_RELEASE);
        fprintf(stderr, "yrss: context closed after a GPU timeout: not drained, device memory "
                        "left to process exit\n");
        for (uint32_t r = 0; r < c->nranges; ++r)
            host_reg_poison(c->range_base[r]);
        delete[] c->w.out;
        delete[] c->w.last_out;
        delete c;   // (shim_win stays: it may be registered for the GPU to read)
        return;
    }
    if (c->w.on) {
        (void)worker_halt(c);
        worker_free(c);
    }
    c->pend.active = false;   // its outputs are abandoned with the context
    // device dispatches may still run on the caller's streams: drain the
    // device before the workspace goes
    (void)hipDeviceSynchronize();
    for (auto &p : c->ev_pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (auto e : c->ev_free)
        (void)hipEventDestroy(e);
    free_burst(c);
    list_ws_free(c->ws);
    (void)hipHostFree(c->d_fault_rec);
    (void)hipFree(c->d_kni);
    (void)hipFree(c->d_fault);
    (void)hipHostFree(c->h_fault);
    (void)hipHostFree(c->h_done);
    for (uint32_t r = 0; r < c->nranges; ++r)
        host_reg_release(c->range_base[r]);
    free(c->shim_win);
    if (c->switch_ev)
        (void)hipEventDestroy(c->switch_ev);
    if (c->stream)
        (void)hipStreamDestroy(c->stream);
    delete c;
}

uint32_t yrss_grid_for(yrss_ctx *c, uint32_t n) { return c ? grid_for(c, n) : 0u; }

int yrss_set_kni(yrss_ctx *c, int enable, const char *method, const char *tcp_ports,
                 const char *udp_ports)
{
    if (!c)
        return -EINVAL;
    bool accept = false;
    if (method) {
        // ff_config.c:548-553: method must be accept or reject (case-insensitive)
        if (strcasecmp(method, "accept") == 0)
            accept = true;
        else if (strcasecmp(method, "reject") != 0)
            return -EINVAL;
    } else if (enable) {
        return -EINVAL;                      // ff_config.c:543-546
    }
    memset(c->kni_bm, 0, sizeof(c->kni_bm));
    kni_parse_ports(tcp_ports, c->kni_bm);
    kni_parse_ports(udp_ports, c->kni_bm + 8192);
    c->kni_enable = enable != 0;
    c->kni_accept = accept;
    YRSS_HIP(hipSetDevice(c->device));
    YRSS_HIP(hipMemcpy(c->d_kni, c->kni_bm, sizeof(c->kni_bm), hipMemcpyHostToDevice));
    YRSS_HIP(hipDeviceSynchronize());   // ordered before any stream's next dispatch
    return 0;
}

int yrss_dispatch_dev_ex(yrss_ctx *c, const struct yrss_dev_batch *b, void *stream)
{
    if (!c || !b)
        return -EINVAL;
    if (c->pend.active)      // the host burst in flight owns the workspace
        return -EBUSY;
    return dispatch_dev_impl(c, b, stream);
}

}  // extern "C"

namespace {

int dispatch_dev_impl(yrss_ctx *c, const struct yrss_dev_batch *b, void *stream)
{
    const uint32_t n = b->n, win_stride = b->win_stride;
    if (win_stride < YRSS_WIN_MIN || (win_stride & 15u) || n > YRSS_MAX_BATCH)
        return -EINVAL;
    if (n && (!b->win || !b->len || !b->q))
        return -EINVAL;
    if (((uintptr_t)b->win & 15u) || ((uintptr_t)b->len & 1u) || ((uintptr_t)b->q & 1u) ||
        ((uintptr_t)b->hash & 3u) || ((uintptr_t)b->qidx & 3u) || ((uintptr_t)b->qstart & 3u))
        return -EINVAL;
    const bool compact = b->qidx != nullptr;
    const bool filter = b->filter != nullptr;
    if (compact && !b->qstart)
        return -EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        if (compact)
            YRSS_HIP(hipMemsetAsync(b->qstart, 0, (c->nb + 1) * sizeof(uint32_t), s));
        return 0;
    }
    // This context's resident worker holds CUs the batch's full grid needs:
    // retire it first (published tickets stay in the ring; the next worker
    // submit or poll relaunches).
    if (c->w.running) {
        const int rc = worker_halt(c);
        if (rc)
            return rc;
    }

    if (c->last_stream_valid && c->last_stream != s) {
        YRSS_HIP(hipEventRecord(c->switch_ev, c->last_stream));
        YRSS_HIP(hipStreamWaitEvent(s, c->switch_ev, 0));
    }
    c->last_stream = s;
    c->last_stream_valid = true;
    // Up to 4096 packets: one launch of the one-workgroup burst kernel (parse,
    // lists in LDS) instead of parse + scan + scatter, ~10 us less per call
    // (profiles/r01_v26_small_kernel_stats.csv: three launches cost >= 15 us of
    // kernel time however small the batch).  Not timed by yrss_timing_*.
    if (small_ok(c, n) && c->tune.one_launch == 0) {
        SmallParams S;
        memset(&S, 0, sizeof(S));
        S.P.win = b->win;
        S.P.len = b->len;
        S.P.stride = win_stride;
        S.P.n = n;
        S.P.q = b->q;
        S.P.hash = b->hash;
        S.P.filter = b->filter;
        S.qidx = compact ? b->qidx : nullptr;
        S.qstart = compact ? b->qstart : nullptr;
        return small_launch(c, S, filter, false, s);
    }
    yrss_ctx::ListWs &W = c->ws;
    const uint32_t grid = grid_for(c, n);
    const Layout lay = layout_for(c, n, grid);
    const uint64_t pwaves = (uint64_t)grid * (kParseBlock / kWave);
    if (compact && ((uint64_t)lay.nchunk + pwaves - 1) / pwaves * c->nb > kCntWords)
        return -EINVAL;   // layout_for sizes chunks so a wave's count slots fit
    const ScatterLds sl = scatter_lds(c->nb);
    const LinePlan lp = line_plan(c, lay);
    // the line scatter reads q (when the bucket is not packed with the rank)
    // as 16-byte vectors
    const bool ranked = compact && lp.ok && n < kLineMaxPkts &&
                        (lp.packed || ((uintptr_t)b->q & 15u) == 0);
    // a line scatter whose per-bucket arrays cannot hold nb is refused before
    // anything is launched (the kernel's own entry check is the backstop)
    if (ranked && !lp.fits && !c->dbg.skip_line_check)
        return -EINVAL;
    if (ranked && W.rank_cap < n) {
        // the ranks' workspace grows to the largest batch seen; the old one
        // may still be read by a scatter queued on this stream
        if (W.rank) {
            YRSS_HIP(hipStreamSynchronize(s));
            (void)hipFree(W.rank);
            W.rank = nullptr;
            W.rank_cap = 0;
        }
        YRSS_HIP(hipMalloc((void **)&W.rank, (size_t)n * sizeof(uint16_t)));
        W.rank_cap = n;
    }
    // The line scatter's launch, planned before the parse kernel: with
    // in-scatter prefixes (up to kFusedMaxNb buckets) the parse kernel sums
    // the totals and no scan kernel runs.  Fused when the range table fits
    // without costing the scatter a resident workgroup.
    void (*line_fn)(LineParams) = nullptr;
    uint32_t line_grid = 0, line_lds_bytes = lp.lds, rts = 0, rcs = 0;
    bool fused = false;
    if (ranked) {
        const bool nt = c->nb > kListNtBuckets;
        line_fn = lp.groups == 4u
                      ? (lp.packed ? (nt ? yrss_scatter_lines<true, 4, true>
                                         : yrss_scatter_lines<true, 4, false>)
                                   : (nt ? yrss_scatter_lines<false, 4, true>
                                         : yrss_scatter_lines<false, 4, false>))
                      : (lp.packed ? (nt ? yrss_scatter_lines<true, 2, true>
                                         : yrss_scatter_lines<true, 2, false>)
                                   : (nt ? yrss_scatter_lines<false, 2, true>
                                         : yrss_scatter_lines<false, 2, false>));
        // persistent: the resident workgroups, each one contiguous range of
        // spans, never more workgroups than spans
        const uint32_t spans = (uint32_t)(((uint64_t)n + lp.seg - 1) / lp.seg);
        line_grid = std::max(1u, std::min(spans, resident_blocks(c, (const void *)line_fn,
                                                                 kLineBlock, lp.lds)));
        if (c->nb <= kFusedMaxNb && W.tot_acc && c->tune.scan_kernel == 0) {
            // ranges of rcs spans (the last ones may be shorter), rc chunks
            const uint32_t rcs_ = (spans + line_grid - 1) / line_grid;
            const uint32_t g_eff = (spans + rcs_ - 1) / rcs_;
            const uint32_t rc = rcs_ << lp.gshift;
            const uint32_t lds = line_lds(c->nb, lp.gshift, lp.lmax, rc + 1u).words * 4u;
            if (rc % 8u == 0 && rc <= kFusedMaxCols && g_eff <= kFusedMaxRanges &&
                c->nb <= kFusedRows * (kLineBlock / kWave - 1u) && lds <= 160u * 1024u &&
                resident_blocks(c, (const void *)line_fn, kLineBlock, lds) >= g_eff) {
                fused = true;
                rcs = rcs_;
                rts = rc + 1u;
                line_grid = g_eff;
                line_lds_bytes = lds;
            }
        }
    }
    ParseParams P = c->proto;
    P.win = b->win;
    P.len = b->len;
    P.q = b->q;
    P.hash = b->hash;
    P.seg_cnt = compact ? W.seg_cnt : nullptr;
    P.rank = ranked ? W.rank : nullptr;
    P.fault = c->d_fault_rec;
    P.n = n;
    P.stride = win_stride;
    P.chunk = lay.chunk;
    P.nchunk = lay.nchunk;
    P.ncol = lay.ncol;
    P.ct_shift = lay.ct_shift;
    P.filter = b->filter;
    P.kni_bm = c->d_kni;
    P.kni_enable = c->kni_enable ? 1u : 0u;
    P.rank_pack = ranked && lp.packed ? 1u : 0u;
    const uint32_t tset = W.tot_set;
    P.tot_acc = fused ? W.tot_acc + (size_t)tset * c->nb : nullptr;
    P.rbin = fused ? W.rbin + (size_t)tset * kLbMaxWgs * c->nb : nullptr;
    P.rbin_chunks = fused ? rcs << lp.gshift : 0u;
    {
        Timed t(c, YRSS_K_PARSE_HASH);
        hipExtLaunchKernelGGL(pick_parse(ranked ? 2 : compact ? 1 : 0, filter), dim3(grid),
                              dim3(kParseBlock),
                              (uint32_t)parse_lds(filter), s, t.a, t.b, 0, P);
    }
    YRSS_HIP(hipGetLastError());
    if (fused)
        W.tot_set = tset ^ 1u;   // this batch's scatter zeroes it for the next
    if (!compact)
        return 0;
    if (!fused) {
        Timed t(c, YRSS_K_SCAN);
        ScanParams SP;
        SP.cnt = W.seg_cnt;
        SP.off = W.seg_off;
        SP.totals = W.totals;
        SP.status = W.scan_status;
        SP.fault = c->d_fault_rec;
        SP.nchunk = lay.nchunk;
        SP.ncol = lay.ncol;
        SP.sub = lay.ncol % (kScanSub * kScanTile) == 0 ? kScanSub : 1u;
        SP.tiles = lay.ncol / (kScanTile * SP.sub);
        if ((++W.scan_epoch & 0x7fffffffu) == 0)   // 0 is the never-published state
            ++W.scan_epoch;
        SP.epoch = W.scan_epoch;
        hipExtLaunchKernelGGL(yrss_seg_scan, dim3(c->nb * SP.tiles), dim3(kScanBlock), 0, s,
                              t.a, t.b, 0, SP);
    }
    YRSS_HIP(hipGetLastError());
    if (ranked) {
        LineParams S;
        S.q = b->q;
        S.rank = W.rank;
        S.seg_off = W.seg_off;
        S.totals = W.totals;
        S.qidx = b->qidx;
        S.qstart = b->qstart;
        S.fault = c->d_fault_rec;
        S.n = n;
        S.nq = c->cfg.nb_queues;
        S.nb = c->nb;
        S.nchunk = lay.nchunk;
        S.ncol = lay.ncol;
        S.seg = lp.seg;
        S.gshift = lp.gshift;
        S.cshift = lay.ct_shift + 6u;
        S.lmax = lp.lmax;
        S.xcd = c->tune.scatter_xcd != 0 ? 1u : 0u;
        S.nt = c->nb > kListNtBuckets ? 1u : 0u;
        S.early = c->nb > 16u ? 1u : 0u;
        S.merge = c->dbg.partial_merge;
        S.fused = fused ? 1u : 0u;
        S.cnt = W.seg_cnt;
        S.rbin = nullptr;
        S.rbin_next = nullptr;
        S.rts = rts;
        S.rcs = rcs;
        S.tot_next = nullptr;
        if (fused) {
            S.totals = W.tot_acc + (size_t)tset * c->nb;
            S.tot_next = W.tot_acc + (size_t)(tset ^ 1u) * c->nb;
            S.rbin = W.rbin + (size_t)tset * kLbMaxWgs * c->nb;
            S.rbin_next = W.rbin + (size_t)(tset ^ 1u) * kLbMaxWgs * c->nb;
            S.xcd = 0;   // (ranges in blockIdx order: the kernel ignores it too)
        }
        Timed t(c, YRSS_K_SCATTER);
        hipExtLaunchKernelGGL(line_fn, dim3(line_grid), dim3(kLineBlock), line_lds_bytes, s, t.a,
                              t.b, 0, S);
        YRSS_HIP(hipGetLastError());
        return 0;
    }
    ScatterParams S;
    S.q = b->q;
    S.seg_off = W.seg_off;
    S.totals = W.totals;
    S.qidx = b->qidx;
    S.qstart = b->qstart;
    S.fault = c->d_fault_rec;
    S.n = n;
    S.seg = lay.seg;
    S.nq = c->cfg.nb_queues;
    S.nb = c->nb;
    S.nchunk = lay.nchunk;
    S.ncol = lay.ncol;
    S.gshift = lay.shift;
    S.cshift = lay.ct_shift + 6u;
    S.aux = sl.aux;
    S.stg = sl.stg;
    S.wlds = sl.wlds;
    S.xcd = c->tune.scatter_xcd != 0 ? 1u : 0u;
    {
        // persistent: the resident workgroups only, never more than the spans
        const uint32_t lds = (uint32_t)(sl.wpb * sl.wlds * sizeof(uint32_t));
        const uint32_t spans = (uint32_t)(((uint64_t)n + lay.seg - 1) / lay.seg);
        uint32_t sgrid = (spans + sl.wpb - 1) / sl.wpb;
        void (*fn)(ScatterParams) = yrss_scatter;
        sgrid = std::min(sgrid, resident_blocks(c, (const void *)fn, sl.wpb * kWave, lds));
        Timed t(c, YRSS_K_SCATTER);
        hipExtLaunchKernelGGL(fn, dim3(std::max(sgrid, 1u)), dim3(sl.wpb * kWave), lds, s, t.a,
                              t.b, 0, S);
    }
    YRSS_HIP(hipGetLastError());
    return 0;
}

}  // namespace

extern "C" {

YRSS_LINE_PROF_HOST_FN   // (measurement builds only)

int yrss_dispatch_dev(yrss_ctx *c, const uint8_t *d_win, uint32_t win_stride,
                      const uint16_t *d_len, uint32_t n, int16_t *d_q, uint32_t *d_hash,
                      uint32_t *d_qidx, uint32_t *d_qstart, void *stream)
{
    yrss_dev_batch b;
    b.win = d_win;
    b.win_stride = win_stride;
    b.n = n;
    b.len = d_len;
    b.q = d_q;
    b.hash = d_hash;
    b.qidx = d_qidx;
    b.qstart = d_qstart;
    b.filter = nullptr;
    return yrss_dispatch_dev_ex(c, &b, stream);
}

int yrss_dispatch_frames(yrss_ctx *c, const uint8_t *const *data, const uint16_t *len,
                         uint32_t n, int16_t *out_q, uint32_t *out_hash, uint32_t *out_qidx,
                         uint32_t *out_qstart)
{
    if (!c || (n && (!data || !len || !out_q)))
        return -EINVAL;
    if (n == 0) {
        if (out_qstart)
            memset(out_qstart, 0, (c->nb + 1) * sizeof(uint32_t));
        return 0;
    }
    int rc = begin_burst(c);
    if (rc)
        return rc;
    YRSS_HIP(hipSetDevice(c->device));
    if ((rc = ensure_burst(c, n)) != 0)
        return rc;
    uint32_t maxlen = 0;
    for (uint32_t i = 0; i < n; ++i)
        maxlen = std::max<uint32_t>(maxlen, len[i]);
    const uint32_t W = host_stride(maxlen);
    for (uint32_t i = 0; i < n; ++i) {
        if (i + 16u < n)
            __builtin_prefetch(data[i + 16u]);
        const uint32_t L = len[i];
        memcpy(c->h_win + (size_t)i * W, data[i], L < W ? L : W);
        c->h_len[i] = (uint16_t)L;
    }
    if ((rc = classify_staged(c, n, W, out_q, out_hash, out_qidx, out_qstart, nullptr,
                              false)) != 0)
        return rc;
    return finish_burst(c);
}

int yrss_set_dispatch_ctx(yrss_ctx *c)
{
    std::lock_guard<std::mutex> lk(g_dispatch_mu);
    g_dispatch_ctx = c;
    return 0;
}

}  // extern "C"

namespace {
int worker_submit(yrss_ctx *c, const void *ptrs, const uint16_t *lens, uint32_t n,
                  int16_t *out_q, uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart,
                  uint32_t flags, uint64_t *ticket, uint64_t win = 0, uint32_t stride = 0);

// The shim's packet as a one-packet burst of the context's resident worker:
// its window (the at most YRSS_WIN_FULL bytes the GPU reads) is copied into a
// slot the context registers on first use, so the caller's mbuf need not lie
// in registered memory.  No HIP call per packet: a submit and a spin on the
// burst's completion word.
int shim_worker(yrss_ctx *c, const uint8_t *d, uint16_t len)
{
    if (!c->shim_win) {
        void *m = aligned_alloc(4096, 4096);
        if (!m)
            return -1;
        if (yrss_register_host_memory(c, m, 4096) != 0) {
            free(m);
            return -1;
        }
        c->shim_win = static_cast<uint8_t *>(m);
    }
    memcpy(c->shim_win, d, len < YRSS_WIN_FULL ? len : YRSS_WIN_FULL);
    const uint8_t *p = c->shim_win;
    int16_t q = 0;
    uint64_t t = 0;
    if (worker_submit(c, &p, &len, 1u, &q, nullptr, nullptr, nullptr, kWorkerFrames, &t) != 0 ||
        yrss_worker_poll(c, t, 1) != 0)
        return -1;
    return q;
}
}  // namespace

extern "C" {

// toeplitz_dispatch's own signature (ff_dpdk_if.c:1945-1946), so it can be
// handed to ff_regist_packet_dispatcher unchanged.  Bit-identical to the
// reference.  A context with a resident worker (yrss_worker_start) serves
// each call as a one-packet worker burst; otherwise each call is a one-packet
// launch (yrss_burst_small) and a synchronisation.  Either way the burst hook
// is the fast path.  queue_id and nb_queues are unused, as in the reference.
int yrss_toeplitz_dispatch(void *data, uint16_t len, uint16_t queue_id, uint16_t nb_queues)
{
    (void)queue_id;
    (void)nb_queues;
    std::lock_guard<std::mutex> lk(g_dispatch_mu);
    static bool noted = false;
    if (!noted) {
        // once per process: this path is compatibility, not speed
        noted = true;
        fprintf(stderr, "yrss: note: yrss_toeplitz_dispatch serves ONE packet per GPU round trip, "
                        "9.3-10.8 us per call (~80x the reference toeplitz_dispatch's 118.6 ns/pkt "
                        "on the CPU); hook the RX burst instead: yrss_dispatch_burst / "
                        "yrss_worker_submit (INTEGRATION.md section 3)\n");
    }
    yrss_ctx *c = g_dispatch_ctx;
    if (!c || !data) {
        // the contract's only error channel (ff_api.h:148-166): F-Stack frees the mbuf
        static bool warned = false;
        if (!c && !warned) {
            warned = true;
            fprintf(stderr, "yrss: yrss_toeplitz_dispatch without yrss_set_dispatch_ctx\n");
        }
        return -1;
    }
    const uint8_t *d = static_cast<const uint8_t *>(data);
    if (c->w.on)
        return shim_worker(c, d, len);
    int16_t q = 0;
    if (yrss_dispatch_frames(c, &d, &len, 1u, &q, nullptr, nullptr, nullptr) != 0)
        return -1;
    return q;
}

int yrss_dispatch_burst(yrss_ctx *c, void *const *mbufs, uint32_t n, int16_t *out_q,
                        uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart,
                        uint32_t flags)
{
    if (!c || (n && (!mbufs || !out_q)))
        return -EINVAL;
    if (n == 0) {
        if (out_qstart)
            memset(out_qstart, 0, (c->nb + 1) * sizeof(uint32_t));
        return 0;
    }
    int rc = begin_burst(c);
    if (rc)
        return rc;
    YRSS_HIP(hipSetDevice(c->device));
    uint32_t W = 0;
    if ((rc = gather_mbufs(c, mbufs, n, &W)) != 0)
        return rc;
    const bool wb = (flags & YRSS_F_WRITE_RSS) != 0;
    if ((rc = classify_staged(c, n, W, out_q, out_hash, out_qidx, out_qstart, nullptr, wb)) != 0)
        return rc;
    if (wb)
        c->pend.wb_mbufs = mbufs;
    return end_burst(c, flags);
}

int yrss_register_host_memory(yrss_ctx *c, void *base, size_t len)
{
    if (!c || !base || !len || c->nranges >= YRSS_MAX_HOST_RANGES)
        return -EINVAL;
    YRSS_HIP(hipSetDevice(c->device));
    int hrc = worker_halt(c);   // a running worker has the old range table
    if (hrc)
        return hrc;
    YRSS_HIP(host_reg_acquire(base, len));
    void *dev = nullptr;
    hipError_t e = hipHostGetDevicePointer(&dev, base, 0);
    if (e != hipSuccess) {
        host_reg_release(base);
        return hip_fail("hipHostGetDevicePointer", e);
    }
    HostRange &r = c->ranges[c->nranges];
    r.lo = (uint64_t)(uintptr_t)base;
    r.hi = r.lo + len;
    r.delta = (int64_t)((uintptr_t)dev - (uintptr_t)base);
    c->range_base[c->nranges++] = base;
    return 0;
}

int yrss_unregister_host_memory(yrss_ctx *c, void *base)
{
    if (!c)
        return -EINVAL;
    for (uint32_t r = 0; r < c->nranges; ++r)
        if (c->range_base[r] == base) {
            // a pending worker burst may read mbufs or write outputs there
            if (c->w.on && c->w.pending)
                return -EBUSY;
            YRSS_HIP(hipSetDevice(c->device));
            const int hrc = worker_halt(c);
            if (hrc)
                return hrc;
            host_reg_release(base);
            for (uint32_t k = r + 1; k < c->nranges; ++k) {
                c->ranges[k - 1] = c->ranges[k];
                c->range_base[k - 1] = c->range_base[k];
            }
            --c->nranges;
            return 0;
        }
    return -EINVAL;
}

namespace {

// Device-visible alias of host bytes [p, p+bytes) if they lie in a registered
// range, else nullptr.
const void *dev_alias(const yrss_ctx *c, const void *p, size_t bytes)
{
    const uint64_t a = (uint64_t)(uintptr_t)p;
    for (uint32_t r = 0; r < c->nranges; ++r)
        if (a >= c->ranges[r].lo && a + bytes <= c->ranges[r].hi)
            return (const void *)(uintptr_t)(a + c->ranges[r].delta);
    return nullptr;
}

int zc_dispatch(yrss_ctx *c, const void *ptrs, const uint16_t *lens, uint32_t n, bool frames,
                int16_t *out_q, uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart,
                uint32_t flags)
{
    const yrss_mbuf_layout &ml = c->cfg.mbuf;
    if (!frames && (ml.off_buf_addr % 8u || ml.off_buf_addr + 8u > 64u || ml.off_data_off % 2u ||
                    ml.off_data_off + 2u > 64u || ml.off_data_len % 2u ||
                    ml.off_data_len + 2u > 64u || ml.off_hash_rss % 4u))
        return -EINVAL;                      // header fields must sit in the first 64 bytes
    if (n == 0) {
        if (out_qstart)
            memset(out_qstart, 0, (c->nb + 1) * sizeof(uint32_t));
        return 0;
    }
    int rc = begin_burst(c);
    if (rc)
        return rc;
    YRSS_HIP(hipSetDevice(c->device));
    if ((rc = ensure_burst(c, n)) != 0)
        return rc;
    hipStream_t s = c->stream;
    const bool small = small_ok(c, n);
    GatherParams G;
    memset(&G, 0, sizeof(G));
    // The pointer (and length) arrays are read in place when registered; else
    // from the pinned staging, in place too on the small-burst path.
    G.ptrs = (const uint64_t *)dev_alias(c, ptrs, (size_t)n * 8);
    if (!G.ptrs) {
        memcpy(c->h_ptrs, ptrs, (size_t)n * 8);
        if (small) {
            G.ptrs = c->dh_ptrs;
        } else {
            YRSS_HIP(hipMemcpyAsync(c->d_ptrs, c->h_ptrs, (size_t)n * 8, hipMemcpyHostToDevice,
                                    s));
            G.ptrs = c->d_ptrs;
        }
    }
    if (frames) {
        G.lens = (const uint16_t *)dev_alias(c, lens, (size_t)n * 2);
        if (!G.lens) {
            memcpy(c->h_len, lens, (size_t)n * 2);
            if (small) {
                G.lens = c->dh_len;
            } else {
                YRSS_HIP(hipMemcpyAsync(c->d_q, c->h_len, (size_t)n * 2, hipMemcpyHostToDevice,
                                        s));
                G.lens = (const uint16_t *)c->d_q;   // d_q is free until the parse kernel
            }
        }
    }
    G.win = c->d_win;
    G.len = c->d_len;
    G.hash = c->d_hash;
    G.n = n;
    G.frames = frames ? 1u : 0u;
    G.nranges = c->nranges;
    G.off_buf_addr = ml.off_buf_addr;
    G.off_data_off = ml.off_data_off;
    G.off_data_len = ml.off_data_len;
    G.off_hash_rss = ml.off_hash_rss;
    memcpy(G.ranges, c->ranges, sizeof(G.ranges));
    const bool compact = out_qidx && out_qstart;
    const bool want_hash = out_hash || (flags & YRSS_F_WRITE_RSS);
    PendingBurst &p = c->pend;
    p = PendingBurst{};
    p.n = n;
    p.outs[0] = {out_q, c->h_q, (size_t)n * 2, false};
    p.outs[1] = {out_hash, c->h_hash, (size_t)n * 4, false};
    p.outs[2] = {compact ? out_qidx : nullptr, c->h_qidx, (size_t)n * 4, false};
    p.outs[3] = {compact ? out_qstart : nullptr, c->h_qstart, (c->nb + 1) * 4, false};
    p.gather_fault = true;
    for (int k = 0; k < 4; ++k)
        p.outs[k].direct = p.outs[k].user && dev_alias(c, p.outs[k].user, p.outs[k].bytes);
    if (small) {
        // one launch: gather + parse + lists, outputs straight to host memory
        // (the caller's arrays when registered, else the pinned staging)
        *c->h_fault = 0;
        G.fault = c->dh_fault;
        SmallParams S;
        memset(&S, 0, sizeof(S));
        S.G = G;
        S.gather = 1;
        S.writeback = (!frames && (flags & YRSS_F_WRITE_RSS)) ? 1u : 0u;
        S.P.win = c->d_win;
        S.P.len = c->d_len;
        S.P.stride = YRSS_WIN_FULL;
        S.P.n = n;
        void *staged[4] = {c->dh_q, c->dh_hash, c->dh_qidx, c->dh_qstart};
        void *dst[4] = {nullptr, nullptr, nullptr, nullptr};
        for (int k = 0; k < 4; ++k)
            if (p.outs[k].user)
                dst[k] = p.outs[k].direct
                             ? const_cast<void *>(dev_alias(c, p.outs[k].user, p.outs[k].bytes))
                             : staged[k];
        S.P.q = (int16_t *)dst[0];
        S.P.hash = (uint32_t *)dst[1];   // the kernel keeps every hash for the write-back
        S.qidx = (uint32_t *)dst[2];
        S.qstart = (uint32_t *)dst[3];
        if ((rc = small_launch(c, S, false)) != 0)
            return rc;
        p.active = true;
        return 0;
    }
    YRSS_HIP(hipMemsetAsync(c->d_fault, 0, sizeof(uint32_t), s));
    G.fault = c->d_fault;
    const uint32_t blocks = std::min<uint32_t>((n + 63u) / 64u, (uint32_t)c->cus * 8u);
    hipLaunchKernelGGL(yrss_gather_zc, dim3(blocks), dim3(256), 0, s, G);
    YRSS_HIP(hipGetLastError());
    yrss_dev_batch b;
    b.win = c->d_win;
    b.win_stride = YRSS_WIN_FULL;
    b.n = n;
    b.len = c->d_len;
    b.q = c->d_q;
    b.hash = want_hash ? c->d_hash : nullptr;
    b.qidx = compact ? c->d_qidx : nullptr;
    b.qstart = compact ? c->d_qstart : nullptr;
    b.filter = nullptr;
    if ((rc = dispatch_dev_impl(c, &b, s)) != 0)
        return rc;
    if (!frames && (flags & YRSS_F_WRITE_RSS)) {
        hipLaunchKernelGGL(yrss_writeback_zc, dim3((n + 255u) / 256u), dim3(256), 0, s, G);
        YRSS_HIP(hipGetLastError());
    }
    const void *src[4] = {c->d_q, c->d_hash, c->d_qidx, c->d_qstart};
    YRSS_HIP(hipMemcpyAsync(c->h_fault, c->d_fault, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    for (int k = 0; k < 4; ++k) {
        if (!p.outs[k].user)
            continue;
        YRSS_HIP(hipMemcpyAsync(p.outs[k].direct ? p.outs[k].user : p.outs[k].stage, src[k],
                                p.outs[k].bytes, hipMemcpyDeviceToHost, s));
    }
    p.dev_fault = compact;
    p.active = true;
    return 0;
}

}  // namespace

int yrss_dispatch_burst_zc(yrss_ctx *c, void *const *mbufs, uint32_t n, int16_t *out_q,
                           uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart,
                           uint32_t flags)
{
    if (!c || (n && (!mbufs || !out_q)))
        return -EINVAL;
    const int rc = zc_dispatch(c, mbufs, nullptr, n, false, out_q, out_hash, out_qidx,
                               out_qstart, flags);
    return rc ? rc : end_burst(c, flags);
}

int yrss_dispatch_frames_zc_ex(yrss_ctx *c, const uint8_t *const *data, const uint16_t *len,
                               uint32_t n, int16_t *out_q, uint32_t *out_hash,
                               uint32_t *out_qidx, uint32_t *out_qstart, uint32_t flags)
{
    if (!c || (n && (!data || !len || !out_q)) || (flags & ~YRSS_F_ASYNC))
        return -EINVAL;
    const int rc = zc_dispatch(c, data, len, n, true, out_q, out_hash, out_qidx, out_qstart,
                               flags);
    return rc ? rc : end_burst(c, flags);
}

int yrss_dispatch_frames_zc(yrss_ctx *c, const uint8_t *const *data, const uint16_t *len,
                            uint32_t n, int16_t *out_q, uint32_t *out_hash, uint32_t *out_qidx,
                            uint32_t *out_qstart)
{
    return yrss_dispatch_frames_zc_ex(c, data, len, n, out_q, out_hash, out_qidx, out_qstart, 0);
}

int yrss_wait(yrss_ctx *c)
{
    if (!c)
        return -EINVAL;
    YRSS_HIP(hipSetDevice(c->device));
    return finish_burst(c);
}

int yrss_route_burst(yrss_ctx *c, void *const *mbufs, uint32_t n, uint16_t queue_id,
                     int kni_primary, const struct yrss_route_ops *ops, void **out_local,
                     void **out_kni, struct yrss_route_result *res)
{
    if (!c || !ops || !ops->enqueue || !ops->clone || !ops->release || !res ||
        (n && (!mbufs || !out_local || !out_kni)))
        return -EINVAL;
    memset(res, 0, sizeof(*res));
    if (n == 0)
        return 0;
    int rc = begin_burst(c);
    if (rc)
        return rc;
    YRSS_HIP(hipSetDevice(c->device));
    uint32_t W = 0;
    if ((rc = gather_mbufs(c, mbufs, n, &W)) != 0)
        return rc;
    std::vector<int16_t> q(n);
    std::vector<int8_t> fc(n);
    std::vector<uint32_t> qidx(n), qstart(c->nb + 1);
    rc = classify_staged(c, n, W, q.data(), nullptr, qidx.data(), qstart.data(), fc.data(),
                         false);
    if (rc == 0)
        rc = finish_burst(c);
    if (rc)
        return rc;
    const uint32_t nq = c->cfg.nb_queues;
    const bool local_ok = queue_id < nq;

    // ARP packets kept on this lcore are deep-cloned to every other queue
    // (ff_dpdk_if.c:1099-1119), in packet order, queue order inside a packet,
    // then once more for KNI when enabled in the primary (:1123-1129).
    std::vector<uint32_t> arp;               // packet indices, ascending
    if (local_ok)
        for (uint32_t k = qstart[queue_id]; k < qstart[queue_id + 1]; ++k)
            if (fc[qidx[k]] == YRSS_FILTER_ARP)
                arp.push_back(qidx[k]);
    std::vector<void *> clones((size_t)arp.size() * nq, nullptr);
    std::vector<void *> kni_clone(arp.size(), nullptr);
    for (size_t a = 0; a < arp.size(); ++a) {
        void *m = mbufs[arp[a]];
        for (uint16_t j = 0; j < nq; ++j)
            if (j != queue_id)
                clones[a * nq + j] = ops->clone(ops->user, m, j);
        if (c->kni_enable && kni_primary)
            kni_clone[a] = ops->clone(ops->user, m, 0xFFFFu);
    }

    // One FIFO burst per ring: that queue's packets merged by packet index with
    // the ARP clones (a failed clone enqueues nothing, :1114-1118).
    std::vector<void *> objs;
    for (uint16_t j = 0; j < nq; ++j) {
        if (j == queue_id)
            continue;
        objs.clear();
        uint32_t k = qstart[j];
        const uint32_t e = qstart[j + 1];
        size_t a = 0;
        while (k < e || a < arp.size()) {
            if (a < arp.size() && (k >= e || arp[a] < qidx[k])) {
                if (clones[a * nq + j])
                    objs.push_back(clones[a * nq + j]);
                ++a;
            } else {
                objs.push_back(mbufs[qidx[k++]]);
            }
        }
        unsigned done = objs.empty() ? 0u : ops->enqueue(ops->user, j, objs.data(),
                                                         (unsigned)objs.size());
        if (done > objs.size())
            done = (unsigned)objs.size();
        res->n_ring[j] = done;
        for (size_t r = done; r < objs.size(); ++r) {      // ring full: free (:1090)
            ops->release(ops->user, objs[r]);
            res->n_freed++;
        }
    }
    // ret < 0 || ret >= nb_queues: freed (:1080-1083)
    for (uint32_t k = qstart[nq]; k < qstart[nq + 1]; ++k) {
        ops->release(ops->user, mbufs[qidx[k]]);
        res->n_freed++;
    }
    // Local packets, in order: protocol_filter decides (:1096-1138).
    if (local_ok) {
        size_t a = 0;
        for (uint32_t k = qstart[queue_id]; k < qstart[queue_id + 1]; ++k) {
            const uint32_t i = qidx[k];
            const int f = fc[i];
            if (f == YRSS_FILTER_ARP) {
                if (kni_clone[a])
                    out_kni[res->n_kni++] = kni_clone[a];
                ++a;
                out_local[res->n_local++] = mbufs[i];
                res->n_arp++;
            } else if (f == YRSS_FILTER_TRUNC || f == YRSS_FILTER_LOOP) {
                out_local[res->n_local++] = mbufs[i];
                res->n_unresolved++;
            } else if (c->kni_enable && ((f == YRSS_FILTER_KNI && c->kni_accept) ||
                                         (f == YRSS_FILTER_UNKNOWN && !c->kni_accept))) {
                out_kni[res->n_kni++] = mbufs[i];
            } else {
                out_local[res->n_local++] = mbufs[i];
            }
        }
    }
    return 0;
}

static void rss_check_params(const yrss_ctx *c, uint16_t nb_queues, uint16_t reta_size,
                             uint16_t queueid, RssCheckParams *P)
{
    memset(P, 0, sizeof(*P));
    memcpy(P->kwin, c->proto.kwin, sizeof(P->kwin));
    P->nq = nb_queues;
    P->mask = (uint32_t)((int)reta_size - 1);     // reta_size 0 -> all ones, as in C
    P->queueid = queueid;
}

int yrss_rss_check_dev(yrss_ctx *c, const struct yrss_rss_tuple *d_tuples, uint32_t n,
                       uint16_t nb_queues, uint16_t reta_size, uint16_t queueid, uint8_t *d_ok,
                       uint32_t *d_hash, void *stream)
{
    if (!c || (n && (!d_tuples || !d_ok)) || ((uintptr_t)d_tuples & 3u) ||
        ((uintptr_t)d_hash & 3u))
        return -EINVAL;
    if (n == 0)
        return 0;
    RssCheckParams P;
    rss_check_params(c, nb_queues, reta_size, queueid, &P);
    P.tuples = d_tuples;
    P.ok = d_ok;
    P.hash = d_hash;
    P.n = n;
    hipLaunchKernelGGL(yrss_rss_check, dim3((n + 255u) / 256u), dim3(256), 0,
                       (hipStream_t)stream, P);
    YRSS_HIP(hipGetLastError());
    return 0;
}

int yrss_rss_lport_sweep(yrss_ctx *c, uint32_t faddr, uint32_t laddr, uint16_t fport,
                         uint16_t nb_queues, uint16_t reta_size, uint16_t queueid,
                         uint32_t *bitmap)
{
    if (!c || !bitmap)
        return -EINVAL;
    YRSS_HIP(hipSetDevice(c->device));
    int rc = ensure_burst(c, 2048);
    if (rc)
        return rc;
    RssCheckParams P;
    rss_check_params(c, nb_queues, reta_size, queueid, &P);
    P.sweep = 1;
    P.fixed[0] = faddr;
    P.fixed[1] = laddr;
    P.fixed[2] = fport;
    P.bitmap = c->d_qidx;                     // 8 KiB of the burst staging
    hipLaunchKernelGGL(yrss_rss_check, dim3(65536 / 256), dim3(256), 0, c->stream, P);
    YRSS_HIP(hipGetLastError());
    YRSS_HIP(hipMemcpyAsync(c->h_qidx, c->d_qidx, 2048 * 4, hipMemcpyDeviceToHost, c->stream));
    YRSS_HIP(hipStreamSynchronize(c->stream));
    memcpy(bitmap, c->h_qidx, 2048 * 4);
    return 0;
}

int yrss_synth_dev(yrss_ctx *c, const struct yrss_synth_params *p, uint64_t first, uint32_t n,
                   uint8_t *d_win, uint32_t win_stride, uint16_t *d_len, void *stream)
{
    if (!c || !p || p->profile >= YRSS_SYN_NPROFILES)
        return -EINVAL;
    if (win_stride < YRSS_WIN_MIN || (win_stride & 15u) || ((uintptr_t)d_win & 15u))
        return -EINVAL;
    if (n == 0)
        return 0;
    hipLaunchKernelGGL(yrss_synth, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       *p, first, n, d_win, win_stride, d_len);
    YRSS_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"

namespace {

void worker_free(yrss_ctx *c)
{
    auto &w = c->w;
    (void)hipHostFree(w.slots);
    (void)hipHostFree(w.done);
    (void)hipFree(w.fault);
    (void)hipFree(w.brec);
    (void)hipHostFree(w.srec);
    (void)hipHostFree(w.ptrs);
    (void)hipHostFree(w.lens);
    (void)hipHostFree(w.q);
    (void)hipHostFree(w.hash);
    (void)hipHostFree(w.qidx);
    (void)hipHostFree(w.qstart);
    (void)hipHostFree(w.next);
    (void)hipHostFree(w.ctl);
    (void)hipFree(w.win);
    (void)hipFree(w.len);
    if (w.stream)
        (void)hipStreamDestroy(w.stream);
    delete[] w.out;
    delete[] w.last_out;
    w = yrss_ctx::WorkerState{};
}

// Ask a running worker launch to leave and wait for it.  Every workgroup
// polls the stop word between bursts; tickets already published stay in the
// ring and are served by the next launch.
int worker_halt(yrss_ctx *c)
{
    auto &w = c->w;
    if (!w.running)
        return 0;
    __atomic_store_n(&w.ctl->stop, 1u, __ATOMIC_RELEASE);
    const hipError_t e = hipStreamSynchronize(w.stream);
    __atomic_store_n(&w.ctl->stop, 0u, __ATOMIC_RELEASE);
    __atomic_store_n(&w.ctl->exited, 0u, __ATOMIC_RELAXED);
    w.running = false;
    return e == hipSuccess ? 0 : hip_fail("worker halt", e);
}

int worker_launch(yrss_ctx *c)
{
    auto &w = c->w;
    WorkerParams W;
    memset(&W, 0, sizeof(W));
    W.P = c->proto;
    W.P.fault = nullptr;   // per burst: W.brec, then the slot's srec entry
    W.P.kni_bm = c->d_kni;
    W.P.kni_enable = 0;
    const yrss_mbuf_layout &ml = c->cfg.mbuf;
    W.G.nranges = c->nranges;
    W.G.off_buf_addr = ml.off_buf_addr;
    W.G.off_data_off = ml.off_data_off;
    W.G.off_data_len = ml.off_data_len;
    W.G.off_hash_rss = ml.off_hash_rss;
    memcpy(W.G.ranges, c->ranges, sizeof(W.G.ranges));
    W.slots = w.d_slots;
    W.done = w.d_done;
    W.fault = w.fault;
    W.brec = w.brec;
    W.srec = w.d_srec;
    W.inject = c->dbg.worker_inject;
    W.ptrs = w.d_ptrs;
    W.lens = w.d_lens;
    W.win = w.win;
    W.len = w.len;
    W.next = w.d_next;
    W.wctl = w.d_ctl;
    W.nslots = w.nslots;
    W.idle_ticks = w.idle_ticks;
    W.life_ticks = w.life_ticks;
    W.poll_sleep = w.poll_sleep;
    hipLaunchKernelGGL(yrss_burst_worker, dim3(w.nblocks), dim3(kSmallBlock),
                       worker_lds(c->nb), w.stream, W);
    YRSS_HIP(hipGetLastError());
    w.running = true;
    return 0;
}

// Keep a launch resident.  A workgroup that leaves (idle ring, lifetime cap)
// counts itself in ctl->exited, a cache hit for the host until the GPU writes
// it: then the rest of that launch is stopped (they leave between bursts) and
// a new one resumes every workgroup at its next ticket.  Retiring the whole
// launch means no workgroup's tickets wait on the others' lifetime.
int worker_ensure(yrss_ctx *c)
{
    auto &w = c->w;
    if (w.running && __atomic_load_n(&w.ctl->exited, __ATOMIC_ACQUIRE) == 0u)
        return 0;
    YRSS_HIP(hipSetDevice(c->device));
    const int rc = worker_halt(c);
    return rc ? rc : worker_launch(c);
}

}  // namespace

extern "C" {

int yrss_worker_start(yrss_ctx *c, uint32_t nslots, uint32_t nblocks)
{
    if (!c || nblocks < 1 || nblocks > YRSS_WORKER_MAX_BLOCKS || nslots < nblocks ||
        nslots > YRSS_WORKER_MAX_SLOTS || nslots % nblocks || c->nb > kSmallMaxNb)
        return -EINVAL;
    if (c->w.on)
        return -EBUSY;
    YRSS_HIP(hipSetDevice(c->device));
    auto &w = c->w;
    w.nslots = nslots;
    w.nblocks = nblocks;
    w.qs_stride = (c->nb + 1u + 15u) & ~15u;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess ||
        khz <= 0)
        khz = 100000;   // s_memrealtime runs at 100 MHz on CDNA
    const char *ei = getenv("YRSS_WORKER_IDLE_MS");
    const char *el = getenv("YRSS_WORKER_LIFE_MS");
    const uint64_t idle_ms = ei ? strtoull(ei, nullptr, 10) : 50u;
    const uint64_t life_ms = el ? strtoull(el, nullptr, 10) : 1000u;
    w.idle_ticks = std::min<uint64_t>(idle_ms, 10000u) * (uint64_t)khz;
    w.life_ticks = std::min<uint64_t>(std::max<uint64_t>(life_ms, 1u), 10000u) * (uint64_t)khz;
    const size_t S = nslots, M = kWorkerMaxBurst;
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipHostMalloc((void **)&w.slots, S * sizeof(WorkerSlot), hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipHostMalloc((void **)&w.done, S * sizeof(uint64_t), hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipMalloc((void **)&w.fault, nblocks * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc((void **)&w.brec, nblocks * 4u * sizeof(uint32_t))) != hipSuccess ||
        (e = hipHostMalloc((void **)&w.srec, S * 4u * sizeof(uint32_t), hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipHostMalloc((void **)&w.next, nblocks * sizeof(uint64_t), hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipHostMalloc((void **)&w.ctl, sizeof(WorkerCtl), hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipHostMalloc((void **)&w.ptrs, S * M * 8u, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void **)&w.lens, S * M * 2u, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void **)&w.q, S * M * 2u, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void **)&w.hash, S * M * 4u, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void **)&w.qidx, S * M * 4u, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void **)&w.qstart, S * w.qs_stride * 4u, hipHostMallocDefault)) !=
            hipSuccess ||
        (e = hipMalloc((void **)&w.win, (size_t)nblocks * M * YRSS_WIN_FULL)) != hipSuccess ||
        (e = hipMalloc((void **)&w.len, (size_t)nblocks * M * 2u)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&w.d_slots, w.slots, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&w.d_done, w.done, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&w.d_srec, w.srec, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&w.d_next, w.next, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&w.d_ctl, w.ctl, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&w.d_ptrs, w.ptrs, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&w.d_lens, w.lens, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&w.d_q, w.q, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&w.d_hash, w.hash, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&w.d_qidx, w.qidx, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&w.d_qstart, w.qstart, 0)) != hipSuccess) {
        worker_free(c);
        return hip_fail("yrss_worker_start", e);
    }
    memset((void *)w.slots, 0, S * sizeof(WorkerSlot));
    memset((void *)w.done, 0, S * sizeof(uint64_t));
    memset((void *)w.srec, 0, S * 4u * sizeof(uint32_t));
    for (uint32_t b = 0; b < nblocks; ++b)
        w.next[b] = b + 1u;            // tickets start at 1; block b serves b+1, b+1+B, ...
    memset((void *)w.ctl, 0, sizeof(WorkerCtl));
    w.out = new yrss_ctx::WorkerState::Out[S];
    w.last_out = new uint64_t[4 * S];
    for (size_t i = 0; i < 4 * S; ++i)
        w.last_out[i] = ~0ull;   // no previous burst: never "same"

    for (size_t i = 0; i < S; ++i)
        w.out[i] = yrss_ctx::WorkerState::Out{nullptr, nullptr, nullptr, nullptr, 0u, true, 0u};
    w.issued = 0;
    w.on = true;
    return 0;
}

}  // extern "C"

namespace {

int worker_submit(yrss_ctx *c, const void *ptrs, const uint16_t *lens, uint32_t n,
                  int16_t *out_q, uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart,
                  uint32_t flags, uint64_t *ticket, uint64_t win, uint32_t stride)
{
    auto &w = c->w;
    if (!w.on)
        return -ENODEV;
    if (n > kWorkerMaxBurst)
        return -E2BIG;
    const uint64_t t = w.issued + 1u;
    const uint32_t si = (uint32_t)(t % w.nslots);
    if (!w.out[si].collected)
        return -EBUSY;   // the slot's previous ticket was not polled yet
    WorkerSlot *sl = w.slots + si;
    if (ptrs)
        memcpy(w.ptrs + (size_t)si * kWorkerMaxBurst, ptrs, (size_t)n * 8u);
    sl->win = win;
    sl->stride = stride;
    if (lens)
        memcpy(w.lens + (size_t)si * kWorkerMaxBurst, lens, (size_t)n * 2u);
    // Outputs the caller keeps in registered memory are written there by the
    // GPU (the poll copies nothing); others go through the slot's staging.
    const size_t base = (size_t)si * kWorkerMaxBurst;
    void *const user[4] = {out_q, out_hash, out_qidx, out_qstart};
    const size_t bytes[4] = {(size_t)n * 2u, (size_t)n * 4u, (size_t)n * 4u,
                             (c->nb + 1u) * 4u};
    void *const stage[4] = {w.d_q + base, w.d_hash + base, w.d_qidx + base,
                            w.d_qstart + (size_t)si * w.qs_stride};
    uint8_t copy = 0;
    bool same = w.last_out != nullptr;
    for (int k = 0; k < 4; ++k) {
        uint64_t d = 0;
        if (user[k]) {
            const uint64_t u = (uint64_t)(uintptr_t)user[k];
            for (uint32_t r = 0; r < c->nranges && !d; ++r)
                if (u >= c->ranges[r].lo && u + bytes[k] <= c->ranges[r].hi)
                    d = u + (uint64_t)c->ranges[r].delta;
            if (!d) {
                d = (uint64_t)(uintptr_t)stage[k];
                copy |= (uint8_t)(1u << k);
            }
        }
        sl->out[k] = d;
        if (same && w.last_out[4 * si + k] != d)
            same = false;
        if (w.last_out)
            w.last_out[4 * si + k] = d;
    }
    sl->n = n;
    sl->flags = flags | (same ? kWorkerSameOut : 0u);
    w.out[si] = yrss_ctx::WorkerState::Out{out_q, out_hash, out_qidx, out_qstart, n, false, copy};
    ++w.pending;
    __atomic_store_n(&sl->seq, t, __ATOMIC_RELEASE);   // n and flags become visible first
    __atomic_store_n(&w.ctl->pub, t, __ATOMIC_RELAXED);  // ring activity (idle is collective)
    w.issued = t;
    *ticket = t;
    const int rc = worker_ensure(c);   // one cached load unless a workgroup left
    if (rc) {
        w.out[si].collected = true;    // no launch serves it: the slot is free again
        --w.pending;
        for (int k = 0; k < 4; ++k)    // and no workgroup cached its addresses
            w.last_out[4 * si + k] = ~0ull;
    }
    return rc;
}

}  // namespace

extern "C" {

int yrss_worker_submit(yrss_ctx *c, void *const *mbufs, uint32_t n, int16_t *out_q,
                       uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart,
                       uint32_t flags, uint64_t *ticket)
{
    if (!c || !ticket || (n && (!mbufs || !out_q)) || (flags & ~YRSS_F_WRITE_RSS))
        return -EINVAL;
    return worker_submit(c, mbufs, nullptr, n, out_q, out_hash, out_qidx, out_qstart, flags,
                         ticket);
}

int yrss_worker_submit_frames(yrss_ctx *c, const uint8_t *const *data, const uint16_t *len,
                              uint32_t n, int16_t *out_q, uint32_t *out_hash,
                              uint32_t *out_qidx, uint32_t *out_qstart, uint64_t *ticket)
{
    if (!c || !ticket || (n && (!data || !len || !out_q)))
        return -EINVAL;
    return worker_submit(c, data, len, n, out_q, out_hash, out_qidx, out_qstart, kWorkerFrames,
                         ticket);
}

int yrss_worker_submit_windows(yrss_ctx *c, const uint8_t *win, uint32_t stride,
                               const uint16_t *len, uint32_t n, int16_t *out_q,
                               uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart,
                               uint64_t *ticket)
{
    if (!c || !ticket || (n && (!win || !len || !out_q)) || stride < YRSS_WIN_MIN ||
        (stride & 15u) || ((uintptr_t)win & 15u))
        return -EINVAL;
    const void *dw = n ? dev_alias(c, win, (size_t)n * stride) : win;
    if (!dw)
        return -EFAULT;   // the windows must lie in registered memory
    return worker_submit(c, nullptr, len, n, out_q, out_hash, out_qidx, out_qstart,
                         kWorkerWindows, ticket, (uint64_t)(uintptr_t)dw, stride);
}

int yrss_worker_poll(yrss_ctx *c, uint64_t ticket, int wait)
{
    if (!c || !c->w.on || ticket == 0 || ticket > c->w.issued)
        return -EINVAL;
    auto &w = c->w;
    const uint32_t si = (uint32_t)(ticket % w.nslots);
    const uint64_t *dn = w.done + si;
    auto &o = w.out[si];
    if (ticket + w.nslots <= w.issued || o.collected)
        return -EINVAL;   // reused or already collected
    uint64_t spins = 0, t0 = 0;
    uint64_t d;
    while (((d = __atomic_load_n(dn, __ATOMIC_ACQUIRE)) & ~kWorkerFlags) != ticket) {
        const int rc = worker_ensure(c);   // a launch that left: relaunch
        if (rc)
            return rc;
        if (!wait)
            return -EAGAIN;
        if ((++spins & 4095u) == 0) {       // a burst takes microseconds: 10 s is a hung GPU
            const uint64_t now = mono_ns();
            if (!t0)
                t0 = now;
            else if (now - t0 > 10ull * 1000000000ull) {
                c->hung = true;   // yrss_fini will not wait for this device
                return -ETIMEDOUT;
            }
        }
        __builtin_ia32_pause();
    }
    o.collected = true;
    --w.pending;
    if (d & kWorkerFault)
        return -EFAULT;
    if (d & kWorkerGuard) {
        // a list guard fired in THIS burst (its record came with done, so no
        // other burst in flight is blamed and nothing waits for the device):
        // logged, and kept in the context's record for yrss_fault_info when
        // that is empty
        const uint32_t *g = w.srec + 4u * si;
        fprintf(stderr, "yrss: device fault %u (%s) in %s at %u (value %u), worker ticket %llu; "
                        "per-queue lists invalid\n",
                g[0], fault_name(g[0]), yrss_kernel_name((int)g[1]), g[2], g[3],
                (unsigned long long)ticket);
        // Claimed the way report_fault claims it on the device (a device batch
        // on another stream may be storing its own record right now): the
        // code word goes 0 -> code by compare-and-swap, and only the winner
        // writes the fields, so a record never mixes two faults.  (A reader
        // between the claim and the field stores sees the code with the
        // previous, cleared fields; take_fault reads after its own sync.)
        uint32_t *r = c->d_fault_rec;
        uint32_t expected = 0u;
        if (__atomic_compare_exchange_n(r, &expected, g[0], false, __ATOMIC_ACQ_REL,
                                        __ATOMIC_ACQUIRE)) {
            __atomic_store_n(r + 1, g[1], __ATOMIC_RELAXED);
            __atomic_store_n(r + 2, g[2], __ATOMIC_RELAXED);
            __atomic_store_n(r + 3, g[3], __ATOMIC_RELEASE);
        }
        return -EIO;
    }
    const size_t base = (size_t)si * kWorkerMaxBurst;
    if (o.copy & 1u)
        memcpy(o.q, w.q + base, (size_t)o.n * 2u);
    if (o.copy & 2u)
        memcpy(o.hash, w.hash + base, (size_t)o.n * 4u);
    if (o.copy & 4u)
        memcpy(o.qidx, w.qidx + base, (size_t)o.n * 4u);
    if (o.copy & 8u)
        memcpy(o.qstart, w.qstart + (size_t)si * w.qs_stride, (c->nb + 1u) * 4u);
    return 0;
}

int yrss_worker_stop(yrss_ctx *c)
{
    if (!c)
        return -EINVAL;
    if (!c->w.on)
        return 0;
    YRSS_HIP(hipSetDevice(c->device));
    const int rc = worker_halt(c);
    worker_free(c);
    return rc;
}

// The context's own work drained: its internal stream and the stream of its
// last device batch (not the whole device: other contexts' streams, and a
// resident worker's, are none of its business, and a hang there must not
// hang this call)
static int sync_ctx(yrss_ctx *c)
{
    YRSS_HIP(hipSetDevice(c->device));
    if (c->stream)
        YRSS_HIP(hipStreamSynchronize(c->stream));
    if (c->last_stream_valid)
        YRSS_HIP(hipStreamSynchronize(c->last_stream));
    return 0;
}

int yrss_status(yrss_ctx *c)
{
    if (!c)
        return -EINVAL;
    const int rc = sync_ctx(c);
    if (rc)
        return rc;
    return take_fault(c) ? -EIO : 0;
}

int yrss_fault_info(yrss_ctx *c, struct yrss_fault *out)
{
    if (!c || !out)
        return -EINVAL;
    const int rc = sync_ctx(c);
    if (rc)
        return rc;
    (void)take_fault(c, out);
    return 0;
}

int yrss_set_tuning(yrss_ctx *c, const struct yrss_tuning *t)
{
    if (!c || !t)
        return -EINVAL;
    const bool pow2 = (t->chunk_tiles & (t->chunk_tiles - 1u)) == 0 &&
                      (t->span_tiles & (t->span_tiles - 1u)) == 0;
    if (!pow2 || t->chunk_tiles > 4096u || t->span_tiles > 65536u || t->parse_blocks > 65536u ||
        t->one_launch > 2u || t->scatter_xcd < -1 || t->scatter_xcd > 1 || t->scan_kernel > 1u)
        return -EINVAL;
    if (c->pend.active)
        return -EBUSY;
    c->tune = *t;
    return 0;
}

#ifdef YRSS_TEST_HOOKS
// Test hooks (include/yrss_test_hooks.h), compiled into libyrss_test.so only:
// libyrss.so has neither these symbols nor the paths they drive
// (tests/test_abi.py checks both libraries).
int yrss_debug_worker_inject(yrss_ctx *c, uint64_t ticket)
{
    if (!c)
        return -EINVAL;
    c->dbg.worker_inject = ticket;   // read at the next worker launch
    return 0;
}

int yrss_debug_line_groups(yrss_ctx *c, uint32_t groups, int skip_host_check)
{
    if (!c || (groups != 0u && groups != 2u && groups != 4u) || skip_host_check < 0 ||
        skip_host_check > 1)
        return -EINVAL;
    c->dbg.line_groups = groups;
    c->dbg.skip_line_check = (uint32_t)skip_host_check;
    return 0;
}

int yrss_debug_partial_merge(yrss_ctx *c, int on)
{
    if (!c || on < 0 || on > 1)
        return -EINVAL;
    c->dbg.partial_merge = (uint32_t)on;
    return 0;
}

#endif

int yrss_timing_enable(yrss_ctx *c, int enable)
{
    if (!c)
        return -EINVAL;
    yrss_timing_read(c, 0, nullptr, nullptr);   // drain pending pairs
    c->timing_mask = (uint32_t)enable & ((1u << YRSS_K_COUNT) - 1u);
    for (int k = 0; k < YRSS_K_COUNT; ++k) {
        c->ms[k] = 0.0;
        c->launches[k] = 0;
        c->durs[k].clear();
    }
    return 0;
}

int yrss_timing_read(yrss_ctx *c, int kernel, double *total_ms, uint32_t *launches)
{
    if (!c || kernel < 0 || kernel >= YRSS_K_COUNT)
        return -EINVAL;
    for (auto &p : c->ev_pending) {
        YRSS_HIP(hipEventSynchronize(p.b));
        float ms = 0.f;
        YRSS_HIP(hipEventElapsedTime(&ms, p.a, p.b));
        c->ms[p.kernel] += ms;
        c->launches[p.kernel] += 1;
        c->durs[p.kernel].push_back(ms);
        c->ev_free.push_back(p.a);
        c->ev_free.push_back(p.b);
    }
    c->ev_pending.clear();
    if (total_ms)
        *total_ms = c->ms[kernel];
    if (launches)
        *launches = c->launches[kernel];
    return 0;
}

int yrss_timing_quantile(yrss_ctx *c, int kernel, double q, double *ms)
{
    if (!c || kernel < 0 || kernel >= YRSS_K_COUNT || !ms || !(q >= 0.0 && q <= 1.0))
        return -EINVAL;
    int rc = yrss_timing_read(c, kernel, nullptr, nullptr);
    if (rc)
        return rc;
    std::vector<float> d = c->durs[kernel];
    if (d.empty())
        return -ENODATA;
    const size_t i = (size_t)(q * (double)(d.size() - 1) + 0.5);
    std::nth_element(d.begin(), d.begin() + (ptrdiff_t)i, d.end());
    *ms = d[i];
    return 0;
}

}  // extern "C"
