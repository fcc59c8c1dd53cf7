// yrss_shard.cpp — multi-GPU sharding helpers for C hosts.
// Host-only; no HIP calls.
//
// A packet's {q, hash} depends only on its own bytes, the key and the config,
// so a batch splits into contiguous shards, one per GPU (one yrss_ctx and one
// stream each), with no collective on the data path.  The reference's
// per-queue rte_ring is FIFO (fs/lib/ff_dpdk_if.c:1087-1093), so the global
// per-queue lists are the per-shard lists concatenated in shard order: the
// only host-side step, done here.  yastack_amd/shard.py is the Python twin.
#include <errno.h>
#include <stdint.h>
#include <string.h>

#include "yrss.h"

extern "C" {

int yrss_shard_range(uint64_t n_total, uint32_t world, uint32_t rank, uint64_t *first,
                     uint64_t *count)
{
    if (world < 1 || rank >= world || !first || !count)
        return -EINVAL;
    const uint64_t base = n_total / world, extra = n_total % world;
    *first = rank * base + (rank < extra ? rank : extra);
    *count = base + (rank < extra ? 1u : 0u);
    return 0;
}

int yrss_merge_queue_lists(uint32_t nshards, uint32_t nbk, const uint64_t *first,
                           const uint32_t *const *qidx, const uint32_t *const *qstart,
                           uint64_t *out_qidx, uint64_t *out_qstart)
{
    if (nshards < 1 || nbk < 1 || nbk > YRSS_MAX_QUEUES + 1 || !first || !qidx || !qstart ||
        !out_qstart)
        return -EINVAL;
    // bucket b's global start = sum over shards of every earlier bucket's count
    out_qstart[0] = 0;
    for (uint32_t b = 0; b < nbk; ++b) {
        uint64_t cnt = 0;
        for (uint32_t s = 0; s < nshards; ++s) {
            if (!qstart[s] || qstart[s][b + 1] < qstart[s][b])
                return -EINVAL;
            cnt += qstart[s][b + 1] - qstart[s][b];
        }
        out_qstart[b + 1] = out_qstart[b] + cnt;
    }
    if (out_qstart[nbk] && !out_qidx)
        return -EINVAL;
    for (uint32_t b = 0; b < nbk; ++b) {
        uint64_t w = out_qstart[b];
        for (uint32_t s = 0; s < nshards; ++s) {
            const uint32_t lo = qstart[s][b], hi = qstart[s][b + 1];
            if (hi > lo && !qidx[s])
                return -EINVAL;
            for (uint32_t k = lo; k < hi; ++k)
                out_qidx[w++] = first[s] + qidx[s][k];
        }
    }
    return 0;
}

}  // extern "C"
