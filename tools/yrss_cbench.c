/*
 * yrss_cbench.c — C host program over the yrss C ABI (include/yrss.h).
 *
 * Measures the host-resident (PCIe-inclusive) soft-RSS rate the way F-Stack
 * would see it: packets sit in a DPDK-layout mbuf pool in host memory
 * (struct rte_mbuf offsets of DPDK 18.02, RTE_MBUF_DEFAULT_BUF_SIZE = 2176,
 * headroom 128), and every burst goes through yrss_dispatch_burst — header
 * gather into pinned memory, H2D, the gfx950 kernels, D2H of queue/hash/
 * per-queue lists.  This is the call that would replace the per-packet
 * dispatcher loop of main_loop_vm_3 (fs/lib/ff_dpdk_if.c:1655-1683).
 *
 *   yrss_cbench [profile] [pool_pkts] [burst] [seconds]
 * prints one JSON line per burst size.  YRSS_CBENCH_MODES picks the paths:
 * 0-3 the one-call burst APIs, 4 the persistent worker, 5 the multi-GPU
 * fan-out (YRSS_CBENCH_FANOUT_DEVICES).
 */
#define _GNU_SOURCE
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <x86intrin.h>

#include "yrss.h"
#include "yrss_synth.h"

#define MBUF_HDR 128u
#define HEADROOM 128u
#define DATAROOM 2048u
#define MBUF_STRIDE (MBUF_HDR + HEADROOM + DATAROOM)   /* 2304: hdr + 2176 buf */

/* data pointer and data_len from each mbuf header (rte_pktmbuf_mtod /
 * rte_pktmbuf_data_len) — the only per-packet host work of the frames path */
static void fill_frames(void *const *m, uint32_t n, const uint8_t **data, uint16_t *len)
{
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t *mb = (const uint8_t *)m[i];
        const uint8_t *buf;
        uint16_t doff;
        memcpy(&buf, mb + YRSS_MBUF_OFF_BUF_ADDR, sizeof(buf));
        memcpy(&doff, mb + YRSS_MBUF_OFF_DATA_OFF, 2);
        memcpy(&len[i], mb + YRSS_MBUF_OFF_DATA_LEN, 2);
        data[i] = buf + doff;
    }
}

/* Placement of the dispatcher thread and of the pool, carried in every JSON
 * line so an outlier explains itself: the CPU the thread runs on (start of the
 * run and at its report), that CPU's NUMA node, the node holding the pool's
 * first and last page.  YRSS_CBENCH_CPU pins the thread before the pool is
 * touched (first touch then places the pool on that CPU's node). */
static int cpu_node(int cpu)
{
    char path[96];
    for (int nd = 0; nd < 64; ++nd) {
        snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/node%d", cpu, nd);
        if (access(path, F_OK) == 0)
            return nd;
    }
    return -1;
}

static int page_node(const void *addr)
{
    int node = -1;
    /* get_mempolicy(&node, NULL, 0, addr, MPOL_F_NODE | MPOL_F_ADDR) */
    if (syscall(SYS_get_mempolicy, &node, NULL, 0UL, addr, 3UL) != 0)
        return -1;
    return node;
}

static int g_cpu_start = -1;
static int g_pool_node[2] = {-1, -1};

static void print_placement(void)
{
    const int cpu = sched_getcpu();
    printf(", \"cpu_start\": %d, \"cpu\": %d, \"cpu_node\": %d, \"pool_node\": [%d, %d]",
           g_cpu_start, cpu, cpu_node(cpu), g_pool_node[0], g_pool_node[1]);
}

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* Persistent worker (yrss_worker_*): `depth` bursts in flight through the
 * ring; the oldest is polled before a slot is reused. */
static int run_worker(const struct yrss_config *cfg0, uint8_t *mem, size_t mem_sz,
                      uint8_t *arena, size_t arena_sz, void **mbufs, uint32_t pool, uint32_t B,
                      double secs, int16_t *q_all, uint32_t *h_all, uint32_t *qi_all,
                      uint32_t profile, int thp, const uint8_t **fdata, uint16_t *flen)
{
    /* YRSS_CBENCH_WORKER_FRAMES: 0 mbuf pointers, 1 (data, data_len) pairs,
     * 2 windows the dispatcher copies into a registered staging ring
     * (yrss_worker_submit_windows) */
    const char *fe = getenv("YRSS_CBENCH_WORKER_FRAMES");
    const int frames = fe ? atoi(fe) : 0;
    if (frames)
        fill_frames(mbufs, pool, fdata, flen);   /* outside the timed region */
    const char *so = getenv("YRSS_CBENCH_WORKER_SLOTOUT");
    const int slotout = so && atoi(so) != 0;
    const char *wn = getenv("YRSS_CBENCH_WIN_NT");
    const int win_nt = wn && atoi(wn) != 0;
    const char *de = getenv("YRSS_CBENCH_WORKER_DEPTH");
    const char *be = getenv("YRSS_CBENCH_WORKER_BLOCKS");
    unsigned blocks = be ? (unsigned)atoi(be) : 4u;
    unsigned depth = de ? (unsigned)atoi(de) : 16u;
    if (blocks < 1 || blocks > YRSS_WORKER_MAX_BLOCKS)
        blocks = 4;
    if (depth < blocks)
        depth = blocks;
    depth = (depth + blocks - 1) / blocks * blocks;
    if ((uint64_t)depth * B > pool || B > YRSS_WORKER_MAX_BURST)
        return 0;
    struct yrss_config cfg = *cfg0;
    cfg.max_burst = 0;
    yrss_ctx *ctx = NULL;
    int rc;
    /* windows form: one staging stretch of B windows per ring slot */
    const size_t wst_sz = frames == 2 ? ((size_t)depth * B * YRSS_WIN_FULL + 4095) & ~(size_t)4095 : 0;
    uint8_t *wst = wst_sz ? aligned_alloc(4096, wst_sz) : NULL;
    if ((rc = yrss_init(&cfg, &ctx)) || (rc = yrss_register_host_memory(ctx, mem, mem_sz)) ||
        (rc = yrss_register_host_memory(ctx, arena, arena_sz)) ||
        (wst && (rc = yrss_register_host_memory(ctx, wst, wst_sz))) ||
        (rc = yrss_worker_start(ctx, depth, blocks))) {
        fprintf(stderr, "worker setup: %d\n", rc);
        return 2;
    }
    static uint32_t qs[YRSS_WORKER_MAX_SLOTS][YRSS_MAX_QUEUES + 2];
    uint64_t *tk = calloc(depth, sizeof(uint64_t));
    uint64_t pkts = 0, i = 0, cyc_poll = 0, cyc_sub = 0, nb = 0;
    uint32_t off = 0;
    double t0 = 0, t1 = 0;
    for (int pass = 0; pass < 2; ++pass) {          /* pass 0: warm-up */
        const double lim = pass ? secs : 0.2;
        t0 = now();
        t1 = t0;
        pkts = 0;
        cyc_poll = cyc_sub = nb = 0;
        while (t1 - t0 < lim) {
            if (off + B > pool)
                off = 0;
            const unsigned k = (unsigned)(i % depth);
            const uint64_t c0 = __rdtsc();
            if (i >= depth && (rc = yrss_worker_poll(ctx, tk[k], 1)) != 0) {
                fprintf(stderr, "worker poll: %d\n", rc);
                return 3;
            }
            const uint64_t c1 = __rdtsc();
            /* YRSS_CBENCH_WORKER_SLOTOUT=1: one fixed output set per ring slot (the
             * F-Stack pattern), else outputs follow the packets through the arena */
            const size_t oo = slotout ? (size_t)k * B : off;
            if (frames == 2) {
                /* the dispatcher's copy of the burst's windows (cache hot after
                 * rte_eth_rx_burst in F-Stack) is part of the timed work */
                uint8_t *w = wst + (size_t)k * B * YRSS_WIN_FULL;
                /* software prefetch 16 windows ahead, into the next burst too
                 * (the cbench pool is cache-cold, unlike headers just received).
                 * YRSS_CBENCH_WIN_NT=1: the staging is written with non-temporal
                 * 16-byte stores, so the dispatcher takes no read-for-ownership
                 * miss on staging lines the GPU read since their last use */
                for (uint32_t j = 0; j < B; ++j) {
                    const uint32_t a = off + j + 16u;
                    if (a < pool) {
                        __builtin_prefetch(fdata[a]);
                        __builtin_prefetch(fdata[a] + 64);
                    }
                    const uint32_t L = flen[off + j] < YRSS_WIN_FULL ? flen[off + j] : YRSS_WIN_FULL;
                    if (win_nt) {
                        /* whole 16-byte pieces: the window's bytes past L are
                         * never read by the GPU (data_len bounds them) */
                        const __m128i *src = (const __m128i *)fdata[off + j];
                        __m128i *dst = (__m128i *)(w + (size_t)j * YRSS_WIN_FULL);
                        for (uint32_t p = 0; p < (L + 15u) / 16u; ++p)
                            _mm_stream_si128(dst + p, _mm_loadu_si128(src + p));
                    } else {
                        memcpy(w + (size_t)j * YRSS_WIN_FULL, fdata[off + j], L);
                    }
                }
                if (win_nt)
                    _mm_sfence();   /* the stores reach memory before the slot is published */
                rc = yrss_worker_submit_windows(ctx, w, YRSS_WIN_FULL, flen + off, B, q_all + oo,
                                                h_all + oo, qi_all + oo, qs[k], &tk[k]);
            } else {
                rc = frames ? yrss_worker_submit_frames(ctx, fdata + off, flen + off, B,
                                                        q_all + oo, h_all + oo, qi_all + oo,
                                                        qs[k], &tk[k])
                            : yrss_worker_submit(ctx, mbufs + off, B, q_all + oo, h_all + oo,
                                                 qi_all + oo, qs[k], 0, &tk[k]);
            }
            cyc_poll += c1 - c0;
            cyc_sub += __rdtsc() - c1;
            ++nb;
            if (rc != 0) {
                fprintf(stderr, "worker submit: %d\n", rc);
                return 3;
            }
            ++i;
            off += B;
            pkts += B;
            if ((i & 63u) == 0)   /* the clock read is not part of a burst's cost */
                t1 = now();
        }
    }
    for (uint64_t j = i > depth ? i - depth : 0; j < i; ++j)
        if ((rc = yrss_worker_poll(ctx, tk[j % depth], 1)) != 0) {
            fprintf(stderr, "worker poll: %d\n", rc);
            return 3;
        }
    t1 = now();
    printf("{\"tool\": \"yrss_cbench\", \"api\": \"%s\", \"profile\": %u, "
           "\"burst\": %u, \"inflight\": %u, \"blocks\": %u, \"pkts\": %llu, "
           "\"seconds\": %.3f, \"mpps\": %.2f, \"us_per_burst\": %.2f, \"thp\": %d, "
           "\"poll_cycles\": %.0f, \"submit_cycles\": %.0f, "
           "\"mode\": 4, \"note\": \"persistent kernel polls a ring of bursts in pinned "
           "memory; %s read over PCIe\"",
           frames == 2 ? "yrss_worker_submit_windows"
           : frames    ? "yrss_worker_submit_frames" : "yrss_worker_submit", profile, B, depth,
           blocks, (unsigned long long)pkts, t1 - t0, pkts / (t1 - t0) / 1e6,
           (t1 - t0) / (pkts / (double)B) * 1e6, thp, nb ? (double)cyc_poll / nb : 0.0,
           nb ? (double)cyc_sub / nb : 0.0,
           frames == 2 ? "contiguous windows the dispatcher copied (one stretch per burst)"
           : frames    ? "windows of (data, data_len) pairs" : "mbuf headers + windows");
    print_placement();
    printf("}\n");
    fflush(stdout);
    free(tk);
    yrss_fini(ctx);
    free(wst);
    return 0;
}

/* Fan-out (yrss_fanout_*): one dispatcher thread, bursts round-robin over the
 * contexts of YRSS_CBENCH_FANOUT_DEVICES (e.g. "0,1,2,3"; default "0"), each
 * with its own worker (`depth` slots, `blocks` workgroups), handed back in
 * submission order; the oldest is taken once every slot is busy. */
static int run_fanout(const struct yrss_config *cfg0, uint8_t *mem, size_t mem_sz,
                      uint8_t *arena, size_t arena_sz, void **mbufs, uint32_t pool, uint32_t B,
                      double secs, int16_t *q_all, uint32_t *h_all, uint32_t *qi_all,
                      uint32_t profile, const uint8_t **fdata, uint16_t *flen)
{
    const char *fe = getenv("YRSS_CBENCH_WORKER_FRAMES");
    const int frames = fe && atoi(fe) != 0;
    if (frames)
        fill_frames(mbufs, pool, fdata, flen);   /* outside the timed region */
    const char *de = getenv("YRSS_CBENCH_WORKER_DEPTH");
    const char *be = getenv("YRSS_CBENCH_WORKER_BLOCKS");
    const char *dv = getenv("YRSS_CBENCH_FANOUT_DEVICES");
    unsigned blocks = be ? (unsigned)atoi(be) : 32u;
    unsigned depth = de ? (unsigned)atoi(de) : 4u * blocks;
    if (blocks < 1 || blocks > YRSS_WORKER_MAX_BLOCKS)
        blocks = 32;
    depth = (depth < blocks ? blocks : depth + blocks - 1) / blocks * blocks;
    int devs[YRSS_FANOUT_MAX_CTX];
    unsigned nd = 0;
    for (const char *p = dv ? dv : "0"; *p && nd < YRSS_FANOUT_MAX_CTX;) {
        devs[nd++] = atoi(p);
        while (*p && *p != ',')
            ++p;
        if (*p == ',')
            ++p;
    }
    const uint64_t inflight = (uint64_t)nd * depth;
    if (inflight * B > pool || B > YRSS_WORKER_MAX_BURST)
        return 0;
    yrss_fanout *f = NULL;
    int rc;
    if ((rc = yrss_fanout_init(cfg0, devs, nd, depth, blocks, &f)) ||
        (rc = yrss_fanout_register_host_memory(f, mem, mem_sz)) ||
        (rc = yrss_fanout_register_host_memory(f, arena, arena_sz))) {
        fprintf(stderr, "fanout setup: %d\n", rc);
        return 2;
    }
    uint32_t(*qs)[YRSS_MAX_QUEUES + 2] = calloc(inflight, sizeof(*qs));
    uint64_t pkts = 0, pkts_all = 0, issued = 0, handed = 0, t;
    uint32_t off = 0;
    double t0 = 0, t1 = 0;
    for (int pass = 0; pass < 2; ++pass) {          /* pass 0: warm-up */
        const double lim = pass ? secs : 0.2;
        t0 = now();
        t1 = t0;
        pkts = 0;
        while (t1 - t0 < lim) {
            if (off + B > pool)
                off = 0;
            if (issued - handed == inflight) {
                if ((rc = yrss_fanout_next(f, 1, &t)) != 0 || t != handed + 1) {
                    fprintf(stderr, "fanout next: %d\n", rc);
                    return 3;
                }
                ++handed;
            }
            const unsigned k = (unsigned)(issued % inflight);
            rc = frames ? yrss_fanout_submit_frames(f, fdata + off, flen + off, B, q_all + off,
                                                    h_all + off, qi_all + off, qs[k], &t)
                        : yrss_fanout_submit(f, mbufs + off, B, q_all + off, h_all + off,
                                             qi_all + off, qs[k], 0, &t);
            if (rc != 0) {
                fprintf(stderr, "fanout submit: %d\n", rc);
                return 3;
            }
            ++issued;
            off += B;
            pkts += B;
            pkts_all += B;
            if ((issued & 63u) == 0)
                t1 = now();
        }
    }
    while (handed < issued) {
        if ((rc = yrss_fanout_next(f, 1, &t)) != 0) {
            fprintf(stderr, "fanout next: %d\n", rc);
            return 3;
        }
        ++handed;
    }
    t1 = now();
    /* Consistency, outside the timed region: every pool position a burst
     * covered holds that burst's q and hash; one context's yrss_dispatch_frames
     * (itself bit-exact against the oracle in the GPU tests) classifies the
     * same frames again and every packet is compared. */
    const uint64_t covered = pkts_all < pool ? pkts_all : (uint64_t)(pool / B) * B;
    uint64_t bad = 0;
    {
        struct yrss_config cfg = *cfg0;
        cfg.max_burst = 4096;
        yrss_ctx *rc_ctx = NULL;
        int16_t *qr = malloc(4096 * sizeof(int16_t));
        uint32_t *hr = malloc(4096 * sizeof(uint32_t));
        if (!frames)
            fill_frames(mbufs, pool, fdata, flen);
        if (!qr || !hr || yrss_init(&cfg, &rc_ctx) != 0) {
            fprintf(stderr, "fanout check setup failed\n");
            return 2;
        }
        for (uint64_t a = 0; a < covered; a += 4096) {
            const uint32_t m = covered - a < 4096 ? (uint32_t)(covered - a) : 4096u;
            if (yrss_dispatch_frames(rc_ctx, fdata + a, flen + a, m, qr, hr, NULL, NULL) != 0) {
                fprintf(stderr, "fanout check dispatch failed\n");
                return 2;
            }
            for (uint32_t i = 0; i < m; ++i)
                bad += qr[i] != q_all[a + i] || hr[i] != h_all[a + i];
        }
        yrss_fini(rc_ctx);
        free(qr);
        free(hr);
    }
    printf("{\"tool\": \"yrss_cbench\", \"api\": \"%s\", \"profile\": %u, "
           "\"burst\": %u, \"gpus\": %u, \"inflight\": %llu, \"blocks\": %u, \"pkts\": %llu, "
           "\"checked\": %llu, \"mismatches\": %llu, "
           "\"seconds\": %.3f, \"mpps\": %.2f, \"mode\": 5, \"note\": \"one dispatcher "
           "thread, bursts round-robin over %u contexts' persistent workers, handed off in "
           "submission order; %s read over PCIe\"",
           frames ? "yrss_fanout_submit_frames" : "yrss_fanout_submit", profile, B, nd,
           (unsigned long long)inflight, blocks, (unsigned long long)pkts,
           (unsigned long long)covered, (unsigned long long)bad, t1 - t0,
           pkts / (t1 - t0) / 1e6, nd, frames ? "windows" : "mbuf headers + windows");
    print_placement();
    printf("}\n");
    fflush(stdout);
    free(qs);
    yrss_fanout_fini(f);
    return bad ? 4 : 0;
}

/* The per-packet registration shim (yrss_toeplitz_dispatch through a
 * dispatch_func_t pointer, as process_packets calls it, ff_dpdk_if.c:1078-1079),
 * one packet at a time over the pool's frames: without a worker (a one-packet
 * launch and a sync per call) and with one resident on the shim's context.
 * Every answer is compared with the burst API's answer for the same packet. */
typedef int (*dispatch_func_t)(void *data, uint16_t len, uint16_t queue_id, uint16_t nb_queues);

static int run_shim(const struct yrss_config *cfg0, void **mbufs, uint32_t pool, double secs,
                    uint32_t profile, const uint8_t **fdata, uint16_t *flen, int16_t *q_all)
{
    struct yrss_config cfg = *cfg0;
    cfg.max_burst = 4096;
    fill_frames(mbufs, pool, fdata, flen);
    dispatch_func_t fn = yrss_toeplitz_dispatch;
    for (int worker = 0; worker < 2; ++worker) {
        yrss_ctx *ctx = NULL;
        int rc;
        if ((rc = yrss_init(&cfg, &ctx)) != 0) {
            fprintf(stderr, "yrss_init: %d\n", rc);
            return 2;
        }
        const uint32_t nref = pool < 4096u ? pool : 4096u;
        if ((rc = yrss_dispatch_frames(ctx, fdata, flen, nref, q_all, NULL, NULL, NULL)) != 0 ||
            (worker && (rc = yrss_worker_start(ctx, 4, 1)) != 0) ||
            (rc = yrss_set_dispatch_ctx(ctx)) != 0) {
            fprintf(stderr, "shim setup: %d\n", rc);
            return 2;
        }
        for (uint32_t j = 0; j < 64; ++j)   /* warm up (first worker call registers its slot) */
            (void)fn((void *)fdata[j], flen[j], 0, 3);
        uint64_t calls = 0, bad = 0;
        const double t0 = now();
        double t1 = t0;
        while (t1 - t0 < secs) {
            const uint32_t j = (uint32_t)(calls % nref);
            const int q = fn((void *)fdata[j], flen[j], 0, 3);
            bad += q != q_all[j];
            ++calls;
            if ((calls & 255u) == 0)
                t1 = now();
        }
        t1 = now();
        printf("{\"tool\": \"yrss_cbench\", \"api\": \"yrss_toeplitz_dispatch\", "
               "\"profile\": %u, \"worker\": %d, \"calls\": %llu, \"seconds\": %.3f, "
               "\"us_per_call\": %.2f, \"mpps\": %.4f, \"mismatches\": %llu, \"mode\": 6, "
               "\"note\": \"per-packet registration shim through a dispatch_func_t pointer; "
               "%s\"}\n",
               profile, worker, (unsigned long long)calls, t1 - t0, (t1 - t0) / calls * 1e6,
               calls / (t1 - t0) / 1e6, (unsigned long long)bad,
               worker ? "one-packet bursts of a resident worker" : "one launch + sync per packet");
        fflush(stdout);
        yrss_set_dispatch_ctx(NULL);
        yrss_fini(ctx);
        if (bad)
            return 4;
    }
    return 0;
}

int main(int argc, char **argv)
{
    const uint32_t profile = argc > 1 ? (uint32_t)atoi(argv[1]) : YRSS_SYN_UDP4;
    const uint32_t pool = argc > 2 ? (uint32_t)atoi(argv[2]) : (1u << 20);
    const uint32_t burst_arg = argc > 3 ? (uint32_t)atoi(argv[3]) : 0;
    const double secs = argc > 4 ? atof(argv[4]) : 2.0;
    const char *cpu_env = getenv("YRSS_CBENCH_CPU");
    if (cpu_env && *cpu_env) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(atoi(cpu_env), &set);
        if (sched_setaffinity(0, sizeof(set), &set) != 0)
            perror("sched_setaffinity");
    }
    g_cpu_start = sched_getcpu();

    /* DPDK mbuf pools live in hugepage memzones; ask for transparent huge pages
     * (YRSS_CBENCH_THP=0 keeps 4 KiB pages) so IOMMU translation for the
     * zero-copy reads sees 2 MiB pages as it would under DPDK */
    const size_t mem_sz = ((size_t)pool * MBUF_STRIDE + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
    const char *thp_env = getenv("YRSS_CBENCH_THP");
    const int thp = !thp_env || atoi(thp_env) != 0;
    uint8_t *mem = mmap(NULL, mem_sz + (2u << 20), PROT_READ | PROT_WRITE,
                        MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (mem == MAP_FAILED)
        mem = NULL;
    else {
        mem = (uint8_t *)(((uintptr_t)mem + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1));
        if (thp)
            madvise(mem, mem_sz, MADV_HUGEPAGE);
    }
    /* burst-side arrays (mbuf pointers as rte_eth_rx_burst fills them, the frame
     * pointer/length pairs, and the outputs) in one page-aligned arena that the
     * zero-copy modes register too, so the GPU reads/writes them in place */
    const size_t arena_sz = ((size_t)pool * (8 + 8 + 2 + 2 + 4 + 4) + 4096 + 4095) & ~(size_t)4095;
    uint8_t *arena = aligned_alloc(4096, arena_sz);
    void **mbufs = (void **)arena;
    const uint8_t **fdata = (const uint8_t **)(arena + (size_t)pool * 8);
    uint16_t *flen = (uint16_t *)(arena + (size_t)pool * 16);
    int16_t *q_all = (int16_t *)(arena + (size_t)pool * 18);
    uint32_t *h_all = (uint32_t *)(arena + (size_t)pool * 20);
    uint32_t *qi_all = (uint32_t *)(arena + (size_t)pool * 24);
    if (!mem || !arena) {
        fprintf(stderr, "out of memory\n");
        return 1;
    }
    struct yrss_synth_params sp = {0x9E3779B97F4A7C15ull, profile, 1u << 20};
    mem[0] = 0;                              /* first touch by this thread */
    for (uint32_t i = 0; i < pool; ++i) {
        uint8_t *m = mem + (size_t)i * MBUF_STRIDE;
        uint8_t *buf = m + MBUF_HDR;
        uint32_t w[20];
        uint16_t len;
        yrss_synth_window(&sp, i, w, &len);
        if (len > DATAROOM)
            len = DATAROOM;
        memset(m, 0, MBUF_HDR);
        memcpy(buf + HEADROOM, w, len < 80 ? len : 80);
        if (len > 80)
            memset(buf + HEADROOM + 80, 0xab, len - 80);
        uint16_t doff = HEADROOM;
        memcpy(m + YRSS_MBUF_OFF_BUF_ADDR, &buf, sizeof(buf));
        memcpy(m + YRSS_MBUF_OFF_DATA_OFF, &doff, 2);
        memcpy(m + YRSS_MBUF_OFF_DATA_LEN, &len, 2);
        mbufs[i] = m;
    }

    g_pool_node[0] = page_node(mem);
    g_pool_node[1] = page_node(mem + mem_sz - 1);
    struct yrss_config cfg;
    yrss_config_default(&cfg);
    const uint32_t bursts[] = {32, 1024, 32768, 1u << 20};
    static const char *names[4] = {"yrss_dispatch_burst", "yrss_dispatch_burst_zc",
                                   "yrss_dispatch_frames_zc", "yrss_dispatch_frames_zc"};
    static const char *notes[4] = {
        "host gathers 64/80-byte windows into pinned memory, H2D, kernels, D2H",
        "GPU reads mbuf headers + windows from registered host memory",
        "host reads data/data_len from each (here cache-cold) mbuf header per burst",
        "data/data_len arrays already built (as after rte_eth_rx_burst, headers hot)"};
    const char *mode_env = getenv("YRSS_CBENCH_MODES");    /* e.g. "13" */
    for (unsigned mode = 0; mode < 4; ++mode)
    for (unsigned bi = 0; bi < sizeof(bursts) / sizeof(bursts[0]); ++bi) {
        const uint32_t B = burst_arg ? burst_arg : bursts[bi];
        if (B > pool || (mode_env && !strchr(mode_env, (int)('0' + mode))))
            continue;
        if (mode == 3)
            fill_frames(mbufs, pool, fdata, flen);    /* outside the timed region */
        cfg.max_burst = B;
        /* YRSS_CBENCH_INFLIGHT=k: k contexts, bursts submitted with YRSS_F_ASYNC
         * round-robin, each context waited on before its next submit */
        const char *inf_env = getenv("YRSS_CBENCH_INFLIGHT");
        unsigned K = inf_env ? (unsigned)atoi(inf_env) : 1u;
        if (K < 1)
            K = 1;
        if (K > 8)
            K = 8;
        if ((uint64_t)K * B > pool)
            K = pool / B ? pool / B : 1;
        const uint32_t aflag = K > 1 ? YRSS_F_ASYNC : 0u;
        yrss_ctx *ctxs[8] = {0};
        int rc = 0;
        for (unsigned k = 0; k < K; ++k) {
            if ((rc = yrss_init(&cfg, &ctxs[k])) != 0) {
                fprintf(stderr, "yrss_init: %d\n", rc);
                return 2;
            }
            if (mode >= 1 && ((rc = yrss_register_host_memory(ctxs[k], mem, mem_sz)) ||
                              (rc = yrss_register_host_memory(ctxs[k], arena, arena_sz)))) {
                fprintf(stderr, "yrss_register_host_memory: %d\n", rc);
                return 2;
            }
        }
        yrss_ctx *ctx = ctxs[0];
        static uint32_t qs[8][YRSS_MAX_QUEUES + 2];
        /* one burst: what the dispatcher lcore would do after rte_eth_rx_burst;
         * outputs land in the burst's own slice of the (registered) arena */
        #define RUN_BURST(cx, k, off) ( \
            mode == 0 ? yrss_dispatch_burst(cx, mbufs + (off), B, q_all + (off), h_all + (off), \
                                            qi_all + (off), qs[k], aflag) : \
            mode == 1 ? yrss_dispatch_burst_zc(cx, mbufs + (off), B, q_all + (off), \
                                               h_all + (off), qi_all + (off), qs[k], aflag) : \
            ((mode == 2 ? fill_frames(mbufs + (off), B, fdata + (off), flen + (off)) : (void)0), \
             yrss_dispatch_frames_zc_ex(cx, fdata + (off), flen + (off), B, q_all + (off), \
                                        h_all + (off), qi_all + (off), qs[k], aflag)))
        /* warm up */
        for (uint32_t off = 0; off + B <= pool && off < 4 * B; off += B)
            if ((rc = RUN_BURST(ctx, 0, off)) != 0 || (rc = yrss_wait(ctx)) != 0) {
                fprintf(stderr, "dispatch: %d\n", rc);
                return 3;
            }
        uint64_t pkts = 0;
        const double t0 = now();
        double t1 = t0;
        uint32_t off = 0;
        uint64_t i = 0;
        int busy[8] = {0};
        while (t1 - t0 < secs) {
            if (off + B > pool)
                off = 0;
            const unsigned k = (unsigned)(i % K);
            if (busy[k] && (rc = yrss_wait(ctxs[k])) != 0) {
                fprintf(stderr, "wait: %d\n", rc);
                return 3;
            }
            rc = RUN_BURST(ctxs[k], k, off);
            if (rc) {
                fprintf(stderr, "dispatch: %d\n", rc);
                return 3;
            }
            busy[k] = K > 1;
            off += B;
            pkts += B;
            ++i;
            t1 = now();
        }
        for (unsigned k = 0; k < K; ++k)
            if (busy[k] && (rc = yrss_wait(ctxs[k])) != 0) {
                fprintf(stderr, "wait: %d\n", rc);
                return 3;
            }
        t1 = now();
        printf("{\"tool\": \"yrss_cbench\", \"api\": \"%s\", \"profile\": %u, "
               "\"burst\": %u, \"inflight\": %u, \"pkts\": %llu, \"seconds\": %.3f, "
               "\"mpps\": %.2f, \"us_per_burst\": %.2f, \"queue_of_first\": %d, \"thp\": %d, "
               "\"mode\": %u, \"note\": \"%s\"}\n",
               names[mode], profile, B, K,
               (unsigned long long)pkts, t1 - t0, pkts / (t1 - t0) / 1e6,
               (t1 - t0) / (pkts / (double)B) * 1e6, q_all[0], thp, mode, notes[mode]);
        fflush(stdout);
        for (unsigned k = 1; k < K; ++k)
            yrss_fini(ctxs[k]);
        yrss_fini(ctx);                 /* also unregisters the pool */
        if (burst_arg)
            break;
    }
    /* YRSS_CBENCH_REPEAT=k: the worker and fan-out runs k times each over the
     * same pool (one JSON line per run: the spread of a placement) */
    const char *rep_env = getenv("YRSS_CBENCH_REPEAT");
    const int reps = rep_env && atoi(rep_env) > 0 ? atoi(rep_env) : 1;
    if (mode_env && strchr(mode_env, '4'))
        for (unsigned bi = 0; bi < 2; ++bi) {
            const uint32_t B = burst_arg ? burst_arg : bursts[bi];
            for (int r = 0; r < reps; ++r) {
                const int rc = run_worker(&cfg, mem, mem_sz, arena, arena_sz, mbufs, pool, B, secs,
                                          q_all, h_all, qi_all, profile, thp, fdata, flen);
                if (rc)
                    return rc;
            }
            if (burst_arg)
                break;
        }
    if (mode_env && strchr(mode_env, '5'))
        for (unsigned bi = 0; bi < 2; ++bi) {
            const uint32_t B = burst_arg ? burst_arg : bursts[bi];
            for (int r = 0; r < reps; ++r) {
                const int rc = run_fanout(&cfg, mem, mem_sz, arena, arena_sz, mbufs, pool, B, secs,
                                          q_all, h_all, qi_all, profile, fdata, flen);
                if (rc)
                    return rc;
            }
            if (burst_arg)
                break;
        }
    if (mode_env && strchr(mode_env, '6')) {
        const int rc = run_shim(&cfg, mbufs, pool, secs, profile, fdata, flen, q_all);
        if (rc)
            return rc;
    }
    free(arena);
    return 0;
}
