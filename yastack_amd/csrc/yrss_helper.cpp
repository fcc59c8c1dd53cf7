// yrss_helper.cpp — the process that owns the GPU for a yrss_remote client
// (include/yrss_remote.h).  Started by the lcore with the ring's memfd as fd
// 3; registers the whole ring with the GPU, starts the persistent worker and
// forwards the ring's bursts to it in ticket order: the GPU reads each slot's
// windows and writes its outputs in place, and the helper publishes
// completion.  If its GPU context faults, this process dies (or stops making
// progress) and the lcore replaces it (yrss_remote_restart); the lcore itself
// never holds a HIP context.
#include <errno.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <deque>
#include <vector>

#include "yrss.h"
#include "yrss_remote_ring.h"

using namespace yrss_ring;

namespace {

struct Pending {
    uint64_t ticket;     // ring ticket
    uint64_t wticket;    // worker ticket
    uint32_t si;
};

void publish(Done *d, uint64_t ticket, int status, Header *h)
{
    d->status = status;
    __atomic_store_n(&d->ticket, ticket, __ATOMIC_RELEASE);
    __atomic_fetch_add(&h->completed, 1u, __ATOMIC_RELEASE);
}

}  // namespace

int main(int argc, char **argv)
{
    int fd = -1;
    for (int i = 1; i + 1 < argc; ++i)
        if (strcmp(argv[i], "--ring-fd") == 0)
            fd = atoi(argv[i + 1]);
    if (fd < 0) {
        fprintf(stderr, "usage: yrss_helper --ring-fd FD (started by yrss_remote_start)\n");
        return 2;
    }
    // Never outlive the lcore.  PR_SET_PDEATHSIG fires when the THREAD that
    // spawned this process exits, which is the lcore process only if that
    // thread is the long-lived lcore thread (yrss_remote.h); the loop below
    // also leaves when the parent process itself is gone (getppid changes).
    prctl(PR_SET_PDEATHSIG, SIGKILL);
    const pid_t parent = getppid();
    if (parent == 1)
        return 3;
    struct stat st;
    if (fstat(fd, &st) != 0 || (size_t)st.st_size < kHeaderBytes)
        return 4;
    const size_t bytes = (size_t)st.st_size;
    void *m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED)
        return 5;
    uint8_t *map = static_cast<uint8_t *>(m);
    Header *h = reinterpret_cast<Header *>(map);
    if (h->magic != kMagic || h->version != kVersion || h->map_bytes != bytes) {
        __atomic_store_n(&h->ready, -EPROTO, __ATOMIC_RELEASE);
        return 6;
    }
    const uint32_t nslots = h->nslots;
    Slot *slots = reinterpret_cast<Slot *>(map + slots_off());
    Done *done = reinterpret_cast<Done *>(map + done_off(nslots));
    const Area a = area(h->max_burst, h->nb);
    auto data = [&](uint32_t si) { return map + h->data_off + (size_t)si * a.bytes; };

    if (h->inject == 1) {
        // fault injection for the CPU tests: a helper that is alive and
        // never completes a burst, as if its GPU hung (no GPU is opened)
        __atomic_store_n(&h->ready, 1, __ATOMIC_RELEASE);
        while (!__atomic_load_n(&h->stop, __ATOMIC_ACQUIRE))
            usleep(1000);
        return 0;
    }

    yrss_ctx *ctx = nullptr;
    yrss_config cfg = h->cfg;
    cfg.max_burst = 0;
    int rc = yrss_init(&cfg, &ctx);
    if (rc == 0)
        rc = yrss_register_host_memory(ctx, map, bytes);
    if (rc == 0)
        rc = yrss_worker_start(ctx, nslots, h->nblocks);
    if (rc != 0) {
        __atomic_store_n(&h->ready, rc < 0 ? rc : -EIO, __ATOMIC_RELEASE);
        if (ctx)
            yrss_fini(ctx);
        return 7;
    }
    __atomic_store_n(&h->ready, 1, __ATOMIC_RELEASE);

    std::deque<Pending> inflight;
    uint64_t next = __atomic_load_n(&h->first, __ATOMIC_ACQUIRE);
    uint32_t idle = 0;
    for (;;) {
        if (__atomic_load_n(&h->stop, __ATOMIC_ACQUIRE))
            break;
        bool busy = false;
        // take published bursts in ticket order (the worker's ring holds at
        // most nslots, as does this one)
        while (inflight.size() < nslots) {
            const uint32_t si = (uint32_t)(next % nslots);
            if (__atomic_load_n(&slots[si].seq, __ATOMIC_ACQUIRE) != next)
                break;
            if (__atomic_load_n(&done[si].ticket, __ATOMIC_ACQUIRE) == next) {
                // completed by the helper this one replaced (a failed submit
                // is published out of order): not re-run, so a client reading
                // its outputs or status never sees them change
                ++next;
                busy = true;
                continue;
            }
            const uint32_t n = slots[si].n;
            uint8_t *d = data(si);
            uint64_t wt = 0;
            // the slot's windows are contiguous (stride 80) in registered
            // memory: the GPU reads them as one stretch
            rc = yrss_worker_submit_windows(
                ctx, d + a.win, kWin, reinterpret_cast<const uint16_t *>(d + a.len), n,
                reinterpret_cast<int16_t *>(d + a.q), reinterpret_cast<uint32_t *>(d + a.hash),
                reinterpret_cast<uint32_t *>(d + a.qidx),
                reinterpret_cast<uint32_t *>(d + a.qstart), &wt);
            if (rc == -EBUSY)
                break;
            if (rc != 0) {
                publish(&done[si], next, rc, h);
            } else {
                inflight.push_back(Pending{next, wt, si});
            }
            ++next;
            busy = true;
        }
        // complete in order
        while (!inflight.empty()) {
            const Pending &p = inflight.front();
            rc = yrss_worker_poll(ctx, p.wticket, 0);
            if (rc == -EAGAIN)
                break;
            publish(&done[p.si], p.ticket, rc, h);
            inflight.pop_front();
            busy = true;
        }
        if (busy || !inflight.empty()) {
            idle = 0;     // bursts on the GPU: keep polling
        } else if (++idle > 4096) {
            usleep(20);   // nothing published for a while: yield the core
            if (getppid() != parent)
                break;    // the lcore process is gone
        }
    }
    yrss_worker_stop(ctx);
    yrss_fini(ctx);
    return 0;
}
