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
 * prints one JSON line per burst size.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "yrss.h"
#include "yrss_synth.h"

#define MBUF_HDR 128u
#define HEADROOM 128u
#define DATAROOM 2048u
#define MBUF_STRIDE (MBUF_HDR + HEADROOM + DATAROOM)   /* 2304: hdr + 2176 buf */

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
    const uint32_t profile = argc > 1 ? (uint32_t)atoi(argv[1]) : YRSS_SYN_UDP4;
    const uint32_t pool = argc > 2 ? (uint32_t)atoi(argv[2]) : (1u << 20);
    const uint32_t burst_arg = argc > 3 ? (uint32_t)atoi(argv[3]) : 0;
    const double secs = argc > 4 ? atof(argv[4]) : 2.0;

    uint8_t *mem = aligned_alloc(64, (size_t)pool * MBUF_STRIDE);
    void **mbufs = malloc(sizeof(void *) * pool);
    if (!mem || !mbufs) {
        fprintf(stderr, "out of memory\n");
        return 1;
    }
    struct yrss_synth_params sp = {0x9E3779B97F4A7C15ull, profile, 1u << 20};
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

    struct yrss_config cfg;
    yrss_config_default(&cfg);
    const uint32_t bursts[] = {32, 1024, 32768, 1u << 20};
    for (unsigned bi = 0; bi < sizeof(bursts) / sizeof(bursts[0]); ++bi) {
        const uint32_t B = burst_arg ? burst_arg : bursts[bi];
        if (B > pool)
            continue;
        cfg.max_burst = B;
        yrss_ctx *ctx = NULL;
        int rc = yrss_init(&cfg, &ctx);
        if (rc) {
            fprintf(stderr, "yrss_init: %d\n", rc);
            return 2;
        }
        int16_t *q = malloc(sizeof(int16_t) * B);
        uint32_t *h = malloc(sizeof(uint32_t) * B);
        uint32_t *qi = malloc(sizeof(uint32_t) * B);
        uint32_t qs[YRSS_MAX_QUEUES + 2];
        /* warm up */
        for (uint32_t off = 0; off + B <= pool && off < 4 * B; off += B)
            if ((rc = yrss_dispatch_burst(ctx, mbufs + off, B, q, h, qi, qs, 0)) != 0) {
                fprintf(stderr, "dispatch: %d\n", rc);
                return 3;
            }
        uint64_t pkts = 0;
        const double t0 = now();
        double t1 = t0;
        uint32_t off = 0;
        while (t1 - t0 < secs) {
            if (off + B > pool)
                off = 0;
            rc = yrss_dispatch_burst(ctx, mbufs + off, B, q, h, qi, qs, 0);
            if (rc) {
                fprintf(stderr, "dispatch: %d\n", rc);
                return 3;
            }
            off += B;
            pkts += B;
            t1 = now();
        }
        printf("{\"tool\": \"yrss_cbench\", \"api\": \"yrss_dispatch_burst\", \"profile\": %u, "
               "\"burst\": %u, \"pkts\": %llu, \"seconds\": %.3f, \"mpps\": %.2f, "
               "\"us_per_burst\": %.2f, \"queue_of_first\": %d}\n",
               profile, B, (unsigned long long)pkts, t1 - t0, pkts / (t1 - t0) / 1e6,
               (t1 - t0) / (pkts / (double)B) * 1e6, q[0]);
        fflush(stdout);
        free(q);
        free(h);
        free(qi);
        yrss_fini(ctx);
        if (burst_arg)
            break;
    }
    free(mbufs);
    free(mem);
    return 0;
}
