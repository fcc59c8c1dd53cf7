/*
 * yrss_remote.h — the soft-RSS engine in a helper process, so that an F-Stack
 * lcore survives a poisoned GPU context.
 *
 * A GPU fault (an illegal address, a hung queue) leaves the HIP context of the
 * process that owns it unusable: every later HIP call fails, and the process
 * cannot be re-executed once it has touched the GPU.  The reference's
 * dispatcher cannot fail this way (fs/lib/ff_dpdk_if.c:1078-1094 is plain C on
 * the lcore), so the lcore that replaces it with the GPU must not own the GPU
 * either.  This client keeps every HIP call out of the lcore:
 *
 *   lcore (this library: no HIP, no GPU)          helper (yrss_helper: libyrss.so)
 *   yrss_remote_submit: copies the burst's   -->  shared ring slot (memfd)  --> persistent
 *   header windows into a ring slot               worker kernel reads the windows in place,
 *   yrss_remote_poll: reads q/hash/lists     <--  writes q/hash/lists into the slot
 *
 * The lcore starts the helper as a child process (posix_spawn; the lcore never
 * opened the GPU, so nothing is re-executed from a GPU process) and watches it:
 * when the helper dies (a GPU fault aborts it, or it is killed) the next poll
 * returns -EPIPE instead of waiting, and yrss_remote_restart starts a fresh
 * helper with a fresh GPU context and republishes every burst still in the
 * ring (their windows are still in the slots), so no burst is lost.  A helper
 * that stops making progress (a hung GPU) makes the poll return -ETIMEDOUT
 * after the context's timeout; yrss_remote_restart then kills and replaces it.
 * The helper dies with its lcore: PR_SET_PDEATHSIG, which fires when the
 * spawning THREAD exits, so call yrss_remote_start and yrss_remote_restart
 * from the long-lived lcore thread, not from a short-lived init or control
 * thread; the helper also leaves once its parent process is gone (it polls
 * getppid() while idle).  A restarted helper re-runs only the tickets not yet
 * completed: a completed ticket's outputs and status never change.
 *
 * Results are bit-identical to yrss_worker_submit_frames (toeplitz_dispatch,
 * ff_dpdk_if.c:1945-2113, and the process_packets FIFO lists, :1058-1094).
 * One client per lcore thread; calls of one client come from one thread.
 */
#ifndef YRSS_REMOTE_H
#define YRSS_REMOTE_H

#include <stdint.h>
#include <sys/types.h>

#include "yrss.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct yrss_remote yrss_remote;

/* Start a helper process for cfg on cfg->device: nslots ring slots of up to
 * max_burst packets (<= YRSS_WORKER_MAX_BURST), served by a persistent worker of
 * nblocks workgroups (yrss_worker_start).  helper_path names the yrss_helper
 * executable (NULL: next to this library).  Waits up to timeout_ms for the
 * helper's GPU initialisation; returns its error (-ENODEV without a GPU, ...)
 * or -ETIMEDOUT.  timeout_ms also bounds every later wait for a burst. */
int yrss_remote_start(const struct yrss_config *cfg, const char *helper_path, uint32_t nslots,
                      uint32_t max_burst, uint32_t nblocks, uint32_t timeout_ms,
                      yrss_remote **out);

/* Queue one burst given as (data pointer, data_len) pairs, as handed over by
 * rte_eth_rx_burst (rte_pktmbuf_mtod / rte_pktmbuf_data_len, ff_dpdk_if.c:
 * 1075-1076): the first min(data_len, YRSS_WIN_FULL) bytes of each packet are
 * copied into the ring slot, so the caller's buffers are free on return.
 * -EBUSY: the slot's previous ticket was not polled yet; -EPIPE: the helper
 * is gone (restart first). */
int yrss_remote_submit(yrss_remote *r, const uint8_t *const *data, const uint16_t *len,
                       uint32_t n, uint64_t *ticket);

/* Results of a ticket: 0 and the outputs copied (any may be NULL; qstart gets
 * nb_queues + 2 words); -EAGAIN not yet (wait = 0); -EPIPE the helper died
 * (the ticket stays queued for yrss_remote_restart); -ETIMEDOUT no completion
 * within the timeout although the helper is alive (a hung GPU); -EIO the
 * helper reported a device-side fault for this burst (yrss_status). */
int yrss_remote_poll(yrss_remote *r, uint64_t ticket, int wait, int16_t *out_q,
                     uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart);

/* Replace the helper (killing it if it still runs) with a fresh one and
 * republish every ticket that was submitted but not completed. */
int yrss_remote_restart(yrss_remote *r);

/* The helper's process id (for monitoring and fault injection in tests). */
pid_t yrss_remote_pid(const yrss_remote *r);

/* Stop the helper and release the ring. */
int yrss_remote_stop(yrss_remote *r);

#ifdef __cplusplus
}
#endif
#endif /* YRSS_REMOTE_H */
