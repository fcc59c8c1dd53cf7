// yrss_remote.cpp — the lcore side of include/yrss_remote.h: a shared ring
// (memfd) and a yrss_helper child process that owns the GPU.  No HIP here:
// the lcore process never opens the GPU, so a device fault kills only the
// helper, and the lcore starts a fresh one (posix_spawn: nothing is
// re-executed from a process that touched the GPU).
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <spawn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "yrss_remote.h"
#include "yrss_remote_ring.h"

extern char **environ;

using namespace yrss_ring;

struct yrss_remote {
    int fd = -1;
    uint8_t *map = nullptr;
    size_t map_bytes = 0;
    Header *hdr = nullptr;
    Slot *slots = nullptr;
    Done *done = nullptr;
    Area area{};
    uint32_t nslots = 0, max_burst = 0, nb = 0;
    uint64_t issued = 0;              // last ticket handed out
    std::vector<uint8_t> collected;   // per slot: its ticket was polled (or none yet)
    std::vector<uint64_t> ticket_of;  // per slot: the ticket it holds
    pid_t pid = -1;
    bool dead = true;
    uint64_t eagain = 0;              // wait = 0 polls that found nothing (liveness every 256)
    uint32_t timeout_ms = 10000;
    std::string helper;
};

namespace {

uint64_t now_ms()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000u + (uint64_t)ts.tv_nsec / 1000000u;
}

std::string default_helper()
{
    Dl_info info;
    if (dladdr((void *)&yrss_remote_start, &info) && info.dli_fname) {
        std::string p(info.dli_fname);
        const size_t s = p.rfind('/');
        return (s == std::string::npos ? std::string(".") : p.substr(0, s)) + "/yrss_helper";
    }
    return "yrss_helper";
}

uint8_t *slot_data(yrss_remote *r, uint32_t si)
{
    return r->map + r->hdr->data_off + (size_t)si * r->area.bytes;
}

// true (and reaped) when the helper has exited
bool helper_gone(yrss_remote *r)
{
    if (r->dead || r->pid <= 0)
        return true;
    int st = 0;
    const pid_t p = waitpid(r->pid, &st, WNOHANG);
    if (p == r->pid || (p < 0 && errno == ECHILD)) {
        r->dead = true;
        r->pid = -1;
        return true;
    }
    return false;
}

void kill_helper(yrss_remote *r)
{
    if (r->pid > 0) {
        kill(r->pid, SIGKILL);
        int st = 0;
        (void)waitpid(r->pid, &st, 0);
    }
    r->pid = -1;
    r->dead = true;
}

// Start a helper on the ring and wait for its GPU initialisation.
int spawn_helper(yrss_remote *r)
{
    Header *h = r->hdr;
    __atomic_store_n(&h->ready, 0, __ATOMIC_RELAXED);
    __atomic_store_n(&h->stop, 0u, __ATOMIC_RELAXED);
    // resume at the oldest ticket not yet done (all of them published)
    uint64_t first = r->issued + 1u;
    for (uint32_t si = 0; si < r->nslots; ++si)
        if (!r->collected[si] && r->ticket_of[si] &&
            __atomic_load_n(&r->done[si].ticket, __ATOMIC_ACQUIRE) != r->ticket_of[si] &&
            r->ticket_of[si] < first)
            first = r->ticket_of[si];
    __atomic_store_n(&h->first, first, __ATOMIC_RELEASE);

    posix_spawn_file_actions_t fa;
    posix_spawn_file_actions_init(&fa);
    posix_spawn_file_actions_adddup2(&fa, r->fd, 3);
    char fdarg[] = "3";
    char *argv[] = {const_cast<char *>(r->helper.c_str()), const_cast<char *>("--ring-fd"), fdarg,
                    nullptr};
    pid_t pid = -1;
    const int e = posix_spawn(&pid, r->helper.c_str(), &fa, nullptr, argv, environ);
    posix_spawn_file_actions_destroy(&fa);
    if (e != 0)
        return -e;
    r->pid = pid;
    r->dead = false;
    const uint64_t t0 = now_ms();
    for (;;) {
        const int32_t rd = __atomic_load_n(&h->ready, __ATOMIC_ACQUIRE);
        if (rd == 1)
            return 0;
        if (rd < 0) {
            kill_helper(r);
            return rd;
        }
        if (helper_gone(r))
            return -EPIPE;
        if (now_ms() - t0 > r->timeout_ms) {
            kill_helper(r);
            return -ETIMEDOUT;
        }
        usleep(200);
    }
}

}  // namespace

extern "C" {

int yrss_remote_start(const struct yrss_config *cfg, const char *helper_path, uint32_t nslots,
                      uint32_t max_burst, uint32_t nblocks, uint32_t timeout_ms,
                      yrss_remote **out)
{
    if (!cfg || !out || nslots < 1 || nblocks < 1 || nslots % nblocks || max_burst < 1 ||
        max_burst > YRSS_WORKER_MAX_BURST || cfg->nb_queues < 1 || cfg->nb_queues > 63 ||
        nslots > YRSS_WORKER_MAX_SLOTS || nblocks > YRSS_WORKER_MAX_BLOCKS)
        return -EINVAL;
    *out = nullptr;
    yrss_remote *r = new yrss_remote();
    r->nslots = nslots;
    r->max_burst = max_burst;
    r->nb = (uint32_t)cfg->nb_queues + 1u;
    r->timeout_ms = timeout_ms ? timeout_ms : 10000u;
    r->helper = helper_path ? helper_path : default_helper();
    r->area = area(max_burst, r->nb);
    r->map_bytes = data_off(nslots) + (size_t)nslots * r->area.bytes;
    r->map_bytes = (r->map_bytes + 4095u) & ~(size_t)4095u;
    r->fd = memfd_create("yrss_ring", MFD_CLOEXEC);
    if (r->fd < 0 || ftruncate(r->fd, (off_t)r->map_bytes) != 0) {
        const int e = errno;
        if (r->fd >= 0)
            close(r->fd);
        delete r;
        return -e;
    }
    void *m = mmap(nullptr, r->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, r->fd, 0);
    if (m == MAP_FAILED) {
        const int e = errno;
        close(r->fd);
        delete r;
        return -e;
    }
    r->map = static_cast<uint8_t *>(m);
    memset(r->map, 0, r->map_bytes);
    r->hdr = reinterpret_cast<Header *>(r->map);
    r->slots = reinterpret_cast<Slot *>(r->map + slots_off());
    r->done = reinterpret_cast<Done *>(r->map + done_off(nslots));
    r->collected.assign(nslots, 1u);
    r->ticket_of.assign(nslots, 0u);
    Header *h = r->hdr;
    h->magic = kMagic;
    h->version = kVersion;
    h->nslots = nslots;
    h->max_burst = max_burst;
    h->nblocks = nblocks;
    h->nb = r->nb;
    h->slot_bytes = r->area.bytes;
    h->data_off = data_off(nslots);
    h->map_bytes = r->map_bytes;
    h->cfg = *cfg;
    if (const char *e = getenv("YRSS_HELPER_INJECT"))   // fault-injection tests only
        h->inject = (uint32_t)atoi(e);
    const int rc = spawn_helper(r);
    if (rc) {
        munmap(r->map, r->map_bytes);
        close(r->fd);
        delete r;
        return rc;
    }
    *out = r;
    return 0;
}

int yrss_remote_submit(yrss_remote *r, const uint8_t *const *data, const uint16_t *len,
                       uint32_t n, uint64_t *ticket)
{
    if (!r || !ticket || n > r->max_burst || (n && (!data || !len)))
        return -EINVAL;
    if (r->dead || ((++r->eagain & 255u) == 0 && helper_gone(r)))   // no syscall per burst
        return -EPIPE;
    const uint64_t t = r->issued + 1u;
    const uint32_t si = (uint32_t)(t % r->nslots);
    if (!r->collected[si])
        return -EBUSY;
    uint8_t *d = slot_data(r, si);
    uint8_t *win = d + r->area.win;
    uint16_t *ln = reinterpret_cast<uint16_t *>(d + r->area.len);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t c = len[i] < kWin ? len[i] : kWin;
        memcpy(win + (size_t)i * kWin, data[i], c);
        ln[i] = len[i];
    }
    r->slots[si].n = n;
    r->collected[si] = 0u;
    r->ticket_of[si] = t;
    __atomic_store_n(&r->slots[si].seq, t, __ATOMIC_RELEASE);
    r->issued = t;
    *ticket = t;
    return 0;
}

int yrss_remote_poll(yrss_remote *r, uint64_t ticket, int wait, int16_t *out_q,
                     uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart)
{
    if (!r || ticket == 0 || ticket > r->issued)
        return -EINVAL;
    const uint32_t si = (uint32_t)(ticket % r->nslots);
    if (r->collected[si] || r->ticket_of[si] != ticket)
        return -EINVAL;
    Done *dn = r->done + si;
    uint64_t t0 = 0, last = 0, spins = 0;
    while (__atomic_load_n(&dn->ticket, __ATOMIC_ACQUIRE) != ticket) {
        // liveness: a helper that died (a GPU fault aborts it) never answers
        if (!wait) {
            if ((++r->eagain & 255u) == 0)
                (void)helper_gone(r);
            return r->dead ? -EPIPE : -EAGAIN;
        }
        if ((++spins & 255u) == 0) {
            if (helper_gone(r))
                return -EPIPE;
            const uint64_t now = now_ms();
            const uint64_t done_n = __atomic_load_n(&r->hdr->completed, __ATOMIC_RELAXED);
            if (!t0 || done_n != last) {   // progress resets the clock
                t0 = now;
                last = done_n;
            } else if (now - t0 > r->timeout_ms) {
                return -ETIMEDOUT;
            }
        }
        __builtin_ia32_pause();
    }
    r->collected[si] = 1u;
    const int st = dn->status;
    if (st)
        return st;
    const uint8_t *d = slot_data(r, si);
    const uint32_t n = r->slots[si].n;
    if (out_q)
        memcpy(out_q, d + r->area.q, (size_t)n * 2u);
    if (out_hash)
        memcpy(out_hash, d + r->area.hash, (size_t)n * 4u);
    if (out_qidx)
        memcpy(out_qidx, d + r->area.qidx, (size_t)n * 4u);
    if (out_qstart)
        memcpy(out_qstart, d + r->area.qstart, ((size_t)r->nb + 1u) * 4u);
    return 0;
}

int yrss_remote_restart(yrss_remote *r)
{
    if (!r)
        return -EINVAL;
    if (!helper_gone(r)) {
        __atomic_store_n(&r->hdr->stop, 1u, __ATOMIC_RELEASE);
        kill_helper(r);
    }
    return spawn_helper(r);
}

pid_t yrss_remote_pid(const yrss_remote *r) { return r ? r->pid : -1; }

int yrss_remote_stop(yrss_remote *r)
{
    if (!r)
        return -EINVAL;
    int rc = 0;
    if (!helper_gone(r)) {
        __atomic_store_n(&r->hdr->stop, 1u, __ATOMIC_RELEASE);
        const uint64_t t0 = now_ms();
        int st = 0;
        for (;;) {
            const pid_t p = waitpid(r->pid, &st, WNOHANG);
            if (p == r->pid) {
                rc = WIFEXITED(st) && WEXITSTATUS(st) == 0 ? 0 : -EIO;
                break;
            }
            if (now_ms() - t0 > r->timeout_ms) {   // a hung helper: kill it
                kill(r->pid, SIGKILL);
                (void)waitpid(r->pid, &st, 0);
                rc = -ETIMEDOUT;
                break;
            }
            usleep(500);
        }
        r->pid = -1;
        r->dead = true;
    }
    munmap(r->map, r->map_bytes);
    close(r->fd);
    delete r;
    return rc;
}

}  // extern "C"
