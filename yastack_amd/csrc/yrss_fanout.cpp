// yrss_fanout.cpp — one dispatcher thread's host bursts fanned out over
// several GPUs (host-resident path).  Host-only: built on the
// public worker ABI (yrss_worker_*), no HIP calls of its own.
//
// The reference's soft dispatch is one lcore: queue 0 polls the NIC and feeds
// every other lcore's dispatch ring (fs/lib/ff_dpdk_if.c:1653-1683, enqueue at
// :1087-1093).  Here that lcore keeps its role and its order: its consecutive
// bursts go round-robin to nctx contexts, each with its own persistent worker
// on its own GPU and PCIe link, and come back in submission order
// (yrss_fanout_next).  Handing each burst's per-queue lists to the rings in that
// order keeps every queue FIFO over the whole stream, as rte_ring does.
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <vector>

#include "yrss.h"

struct yrss_fanout {
    std::vector<yrss_ctx *> ctx;
    uint64_t issued = 0;   // last ticket handed out (tickets start at 1)
    uint64_t handed = 0;   // last ticket returned by yrss_fanout_next
};

extern "C" {

int yrss_fanout_route(uint64_t ticket, uint32_t nctx, uint32_t *ctx, uint64_t *ctx_ticket)
{
    if (ticket == 0 || nctx == 0 || !ctx || !ctx_ticket)
        return -EINVAL;
    *ctx = (uint32_t)((ticket - 1) % nctx);
    *ctx_ticket = (ticket - 1) / nctx + 1;   // each context's worker numbers its own bursts
    return 0;
}

int yrss_fanout_fini(yrss_fanout *f)
{
    if (!f)
        return -EINVAL;
    int rc = 0;
    for (yrss_ctx *c : f->ctx) {
        const int r = yrss_worker_stop(c);
        if (r && !rc)
            rc = r;
        yrss_fini(c);
    }
    delete f;
    return rc;
}

int yrss_fanout_init(const struct yrss_config *cfg, const int *devices, uint32_t nctx,
                     uint32_t nslots, uint32_t nblocks, yrss_fanout **out)
{
    if (!cfg || !devices || !out || nctx < 1 || nctx > YRSS_FANOUT_MAX_CTX)
        return -EINVAL;
    *out = nullptr;
    yrss_fanout *f = new (std::nothrow) yrss_fanout;
    if (!f)
        return -ENOMEM;
    for (uint32_t i = 0; i < nctx; ++i) {
        struct yrss_config c = *cfg;
        c.device = devices[i];
        c.max_burst = 0;   // the worker has its own staging
        yrss_ctx *x = nullptr;
        int rc = yrss_init(&c, &x);
        if (rc == 0 && (rc = yrss_worker_start(x, nslots, nblocks)) != 0)
            yrss_fini(x);
        if (rc) {
            (void)yrss_fanout_fini(f);
            return rc;
        }
        f->ctx.push_back(x);
    }
    *out = f;
    return 0;
}

int yrss_fanout_register_host_memory(yrss_fanout *f, void *base, size_t len)
{
    if (!f)
        return -EINVAL;
    for (size_t i = 0; i < f->ctx.size(); ++i) {
        const int rc = yrss_register_host_memory(f->ctx[i], base, len);
        if (rc) {
            while (i-- > 0)
                (void)yrss_unregister_host_memory(f->ctx[i], base);
            return rc;
        }
    }
    return 0;
}

int yrss_fanout_unregister_host_memory(yrss_fanout *f, void *base)
{
    if (!f)
        return -EINVAL;
    int rc = 0;
    for (yrss_ctx *c : f->ctx) {
        const int r = yrss_unregister_host_memory(c, base);
        if (r && !rc)
            rc = r;
    }
    return rc;
}

static int fanout_submit(yrss_fanout *f, const void *ptrs, const uint16_t *lens, uint32_t n,
                         int16_t *out_q, uint32_t *out_hash, uint32_t *out_qidx,
                         uint32_t *out_qstart, uint32_t flags, uint64_t *ticket)
{
    if (!f || !ticket)
        return -EINVAL;
    const uint64_t g = f->issued + 1;
    uint32_t k;
    uint64_t want;
    (void)yrss_fanout_route(g, (uint32_t)f->ctx.size(), &k, &want);
    uint64_t t = 0;
    const int rc = lens ? yrss_worker_submit_frames(f->ctx[k], (const uint8_t *const *)ptrs, lens,
                                                    n, out_q, out_hash, out_qidx, out_qstart, &t)
                        : yrss_worker_submit(f->ctx[k], (void *const *)ptrs, n, out_q, out_hash,
                                             out_qidx, out_qstart, flags, &t);
    if (rc)
        return rc;   // nothing was queued: the round-robin position stays
    if (t != want)
        return -EPROTO;   // the context was driven outside this fan-out
    f->issued = g;
    *ticket = g;
    return 0;
}

int yrss_fanout_submit(yrss_fanout *f, void *const *mbufs, uint32_t n, int16_t *out_q,
                       uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart,
                       uint32_t flags, uint64_t *ticket)
{
    return fanout_submit(f, mbufs, nullptr, n, out_q, out_hash, out_qidx, out_qstart, flags,
                         ticket);
}

int yrss_fanout_submit_frames(yrss_fanout *f, const uint8_t *const *data, const uint16_t *len,
                              uint32_t n, int16_t *out_q, uint32_t *out_hash,
                              uint32_t *out_qidx, uint32_t *out_qstart, uint64_t *ticket)
{
    if (n && !len)
        return -EINVAL;
    static const uint16_t none = 0;
    return fanout_submit(f, data, len ? len : &none, n, out_q, out_hash, out_qidx, out_qstart,
                         0, ticket);
}

int yrss_fanout_next(yrss_fanout *f, int wait, uint64_t *ticket)
{
    if (!f || !ticket)
        return -EINVAL;
    if (f->handed == f->issued)
        return -ENOENT;
    const uint64_t g = f->handed + 1;
    uint32_t k;
    uint64_t t;
    (void)yrss_fanout_route(g, (uint32_t)f->ctx.size(), &k, &t);
    const int rc = yrss_worker_poll(f->ctx[k], t, wait);
    if (rc == 0 || rc == -EFAULT) {   // -EFAULT: collected, a pointer was out of range
        f->handed = g;
        *ticket = g;
    }
    return rc;
}

uint32_t yrss_fanout_size(yrss_fanout *f)
{
    return f ? (uint32_t)f->ctx.size() : 0u;
}

}  // extern "C"
