/*
 * yrss.h — C ABI of the MI355X software-RSS engine (parse + Toeplitz hash +
 * per-queue dispatch) that replaces yastack / F-Stack's soft-dispatch path.
 *
 * Reference path being replaced (all paths relative to the yastack tree):
 *   fs/lib/ff_api.h:167-174        dispatch_func_t, ff_regist_packet_dispatcher,
 *                                  toeplitz_dispatch prototypes
 *   fs/lib/ff_dpdk_if.c:1881-1902  toeplitz_hash (bit-serial Toeplitz)
 *   fs/lib/ff_dpdk_if.c:1945-2113  toeplitz_dispatch (L2/L3/L4 parse + queue)
 *   fs/lib/ff_dpdk_if.c:1058-1094  process_packets dispatcher block (drop if
 *                                  ret<0 || ret>=nb_queues, else enqueue to
 *                                  dispatch_ring[port][ret])
 *   fs/lib/ff_dpdk_if.c:1653-1683  main_loop_vm_3 RX burst → per-packet loop
 *
 * The reference calls its dispatcher once per packet on the CPU.  This ABI is
 * burst-shaped instead: the hook sits between rte_eth_rx_burst
 * (ff_dpdk_if.c:1655) and the per-packet loop (:1674), classifies a whole
 * batch on the GPU, and returns per-packet {queue, hash} plus per-queue FIFO
 * index lists (the device-side analogue of dispatch_ring[port][q]).
 *
 * Everything here is plain C: pointers, sizes, ints.  No HIP or torch types
 * appear in signatures; device pointers are `void *`/typed pointers to device
 * memory and HIP streams are passed as `void *` (hipStream_t, NULL = default).
 *
 * Errors: every int-returning call returns 0 on success or a negative errno
 * (-EINVAL bad argument, -ENOMEM allocation failure, -ENODEV no usable GPU,
 * -EIO HIP runtime failure).  This mirrors the reference's only error channel
 * (the sign of the dispatcher's return, ff_api.h:160-163) — there is no errno.
 */
#ifndef YRSS_H
#define YRSS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YRSS_VERSION_STRING "yrss 0.1.0 (gfx950)"

/* ---- constants mirrored from the reference -------------------------------- */

/* Toeplitz key length used by the reference: sizeof(default_rsskey_40bytes),
 * fs/lib/ff_dpdk_if.c:113-119. */
#define YRSS_RSS_KEY_LEN 40

/* Default queue returned for every packet the reference does not hash
 * (`uint16_t default_Q = 2`, ff_dpdk_if.c:1948). */
#define YRSS_DEFAULT_Q 2

/* Queue written for a hashed TCP packet whose L4 ports lie beyond the bytes
 * the caller staged in its header window (only possible when win_stride < 78
 * and data_len > win_stride).  Never produced by yrss_dispatch_burst /
 * yrss_dispatch_frames, which always stage enough bytes.  Such packets land
 * in the drop bucket, like any ret outside [0, nb_queues). */
#define YRSS_Q_TRUNCATED (-2)

/* Widest header window the parse ever needs: with IHL=15 the TCP ports sit at
 * bytes 74..77 (14 + 60 + 4).  A window stride >= 80 never truncates. */
#define YRSS_WIN_FULL 80
/* Minimum window stride: one 64-byte coalesced header block per packet. */
#define YRSS_WIN_MIN 64

/* Largest supported values (queues are buckets of the compaction; q is int16;
 * packet indices stay well inside uint32 arithmetic). */
#define YRSS_MAX_QUEUES 256
#define YRSS_MAX_PROCS 4096
#define YRSS_MAX_BATCH (1u << 31)

/* struct rte_mbuf field offsets for the in-tree DPDK 18.02 (x86_64), measured
 * from dpdk/lib/librte_mbuf/rte_mbuf.h:412-560.  The burst API reads
 * buf_addr/data_off/data_len and may write hash.rss; callers on another DPDK
 * version override them in yrss_config.mbuf. */
#define YRSS_MBUF_OFF_BUF_ADDR 0
#define YRSS_MBUF_OFF_DATA_OFF 16
#define YRSS_MBUF_OFF_DATA_LEN 40
#define YRSS_MBUF_OFF_HASH_RSS 44

struct yrss_mbuf_layout {
    uint16_t off_buf_addr;   /* void *buf_addr                         */
    uint16_t off_data_off;   /* uint16_t data_off                      */
    uint16_t off_data_len;   /* uint16_t data_len (first segment only) */
    uint16_t off_hash_rss;   /* uint32_t hash.rss                      */
};

/* ---- configuration --------------------------------------------------------- */

/* The knobs toeplitz_dispatch / process_packets read:
 *   rss_key            default_rsskey_40bytes           ff_dpdk_if.c:113-119
 *   nb_procs           ff_global_cfg.dpdk.nb_procs      ff_config.c:133 (popcount lcore_mask)
 *   soft_dispatch      ff_global_cfg.dpdk.soft_dispatch ff_config.c:440-441
 *   dispatch_only_core ff_global_cfg.system.dispatch_only_core  ff_config.c:450-451
 *   nb_queues          qconf->nb_queue_list[port]       ff_dpdk_if.c:1063, :420
 */
struct yrss_config {
    uint8_t  rss_key[YRSS_RSS_KEY_LEN];
    uint32_t rss_key_len;          /* 4..40; the reference always uses 40   */
    int32_t  nb_procs;             /* 1..YRSS_MAX_PROCS                     */
    uint16_t nb_queues;            /* 1..YRSS_MAX_QUEUES (drop if q>=this)  */
    uint8_t  soft_dispatch;        /* 0/1                                   */
    uint8_t  dispatch_only_core;   /* 0/1; with soft_dispatch needs nb_procs>=2 */
    int32_t  device;               /* HIP device ordinal for yrss_init      */
    uint32_t max_burst;            /* host-burst staging capacity (packets) */
    struct yrss_mbuf_layout mbuf;  /* rte_mbuf offsets for the burst API    */
};

/* Fill cfg with the reference defaults: the Mellanox key, the shipped
 * fs/config/config.ini (lcore_mask=7 → nb_procs=3, soft_dispatch=1,
 * dispatch_only_core=1), nb_queues=nb_procs, device 0, DPDK 18.02 mbuf. */
void yrss_config_default(struct yrss_config *cfg);

/* Validate without touching the GPU.  Rejects what the reference would divide
 * by zero on (dispatch_only_core && soft_dispatch && nb_procs < 2,
 * ff_dpdk_if.c:2031-2032) and out-of-range sizes.  0 or -EINVAL. */
int yrss_config_validate(const struct yrss_config *cfg);

/* ---- context ------------------------------------------------------------------ */

typedef struct yrss_ctx yrss_ctx;

/* Create a context bound to cfg->device: uploads the key schedule, sizes the
 * compaction workspace, allocates pinned staging for max_burst packets.
 * One context per host thread (the reference's dispatcher is single-threaded,
 * ff_dpdk_if.c:1653). */
int  yrss_init(const struct yrss_config *cfg, yrss_ctx **out);
void yrss_fini(yrss_ctx *ctx);

/* ---- device-resident dispatch (the metric path) ------------------------------ */

/* Classify n packets whose header windows already sit in HBM.
 *   d_win      window i at d_win + i*win_stride holds bytes
 *              [0, min(len_i, win_stride)) of packet i's first segment;
 *              16-byte aligned, win_stride % 16 == 0, win_stride >= 64.
 *   d_len      n x uint16 data_len (rte_pktmbuf_data_len, ff_dpdk_if.c:1076)
 *   d_q        n x int16 queue = toeplitz_dispatch's return
 *   d_hash     n x uint32 Toeplitz hash (0 where the reference does not hash);
 *              may be NULL
 *   d_qidx     n x uint32 packet indices grouped by bucket, FIFO inside each
 *              bucket; may be NULL (then d_qstart is ignored)
 *   d_qstart   nb_queues+2 x uint32: bucket b in [0,nb_queues) holds the
 *              packets dispatched to queue b; bucket nb_queues holds the
 *              packets process_packets frees (ret<0 || ret>=nb_queues,
 *              ff_dpdk_if.c:1080-1083).  Bucket b = d_qidx[d_qstart[b] ..
 *              d_qstart[b+1]).  d_qstart[nb_queues+1] == n.
 *   stream     hipStream_t (NULL = legacy default stream)
 * n <= YRSS_MAX_BATCH.  Asynchronous: returns after enqueueing the kernels.
 * Batches of <= 4096 packets (with nb_queues + 1 <= 64) run as one launch of
 * the one-workgroup burst kernel instead of parse + scan + scatter (same
 * outputs; yrss_timing_* does not count it; yrss_tuning.one_launch turns it off).
 * Dispatches of one context share its compaction workspace: a dispatch on a
 * different stream than the context's previous one waits (on the device) for
 * the work already queued there, so streams may be mixed freely; dispatches
 * on one stream pay nothing for this.  yrss_fini drains the device.
 * Stream lifetime: the context remembers the stream of its last device batch
 * (the switch above, and yrss_status / yrss_fault_info synchronise it), so
 * that stream must stay alive until the context's next dispatch on another
 * stream, its next yrss_status / yrss_fault_info, or yrss_fini. */
int yrss_dispatch_dev(yrss_ctx *ctx, const uint8_t *d_win, uint32_t win_stride,
                      const uint16_t *d_len, uint32_t n, int16_t *d_q,
                      uint32_t *d_hash, uint32_t *d_qidx, uint32_t *d_qstart,
                      void *stream);

/* ---- protocol_filter / KNI ----------------------------- */

/* Per-packet protocol_filter class (fs/lib/ff_dpdk_kni.h:34-38 FilterReturn),
 * computed in the same kernel pass as the hash when requested. */
#define YRSS_FILTER_UNKNOWN (-1)
#define YRSS_FILTER_ARP 1
#define YRSS_FILTER_KNI 2
/* Boundary outcomes the reference cannot produce: the IPIP header walk left
 * the staged window, or hit IHL=0 under IPIP, where ff_kni_proto_filter
 * recurses on the same header forever (ff_dpdk_kni.c:274-275). */
#define YRSS_FILTER_TRUNC (-2)
#define YRSS_FILTER_LOOP (-3)

/* Configure KNI exactly as ff_kni_init/init_kni do (ff_dpdk_if.c:597-606,
 * ff_dpdk_kni.c:99-118,300-331): enable, method "accept"/"reject" (anything
 * else is rejected like ff_config.c:548-553), and comma/range port lists
 * ("80,443,8000-8080") parsed with kni_set_bitmap's rules into the 8 KiB
 * htons-indexed bitmaps.  NULL lists leave a bitmap empty. */
int yrss_set_kni(yrss_ctx *ctx, int enable, const char *method,
                 const char *tcp_ports, const char *udp_ports);

/* Full device batch: yrss_dispatch_dev plus the optional filter output. */
struct yrss_dev_batch {
    const uint8_t *win;       /* as d_win of yrss_dispatch_dev          */
    uint32_t win_stride;
    uint32_t n;
    const uint16_t *len;
    int16_t *q;
    uint32_t *hash;           /* may be NULL                            */
    uint32_t *qidx;           /* may be NULL                            */
    uint32_t *qstart;         /* required with qidx                     */
    int8_t *filter;           /* YRSS_FILTER_* per packet, or NULL      */
};
int yrss_dispatch_dev_ex(yrss_ctx *ctx, const struct yrss_dev_batch *b, void *stream);


/* ---- host-resident dispatch (the drop-in burst hook) ------------------------ */

/* Classify a burst of DPDK mbufs straight off rte_eth_rx_burst.
 *   mbufs      n x `struct rte_mbuf *` (read per cfg->mbuf offsets)
 *   out_q      n x int16 host array (required)
 *   out_hash   n x uint32 host array or NULL
 *   out_qidx / out_qstart  host arrays as in yrss_dispatch_dev, or NULL
 *   flags      YRSS_F_WRITE_RSS: also store each hash into mbuf hash.rss
 * Gathers min(data_len, 64 or 80) header bytes into pinned memory.  Bursts of
 * up to 4096 packets (with nb_queues + 1 <= 64) run as ONE kernel launch that
 * reads the pinned windows and writes the pinned results in place; larger ones
 * copy to the GPU, run the batch kernels and copy back.  Synchronous unless
 * flags has YRSS_F_ASYNC. */
#define YRSS_F_WRITE_RSS 0x1u
/* Return once the burst is queued on the context's stream; the outputs (and the
 * hash.rss write-back) are valid after yrss_wait(ctx) returns 0.  Everything
 * the call reads in place (the mbufs, registered pointer/length arrays) and
 * the output arrays must stay untouched until then.  One burst in flight per
 * context: another host-resident call (or yrss_dispatch_dev*) returns -EBUSY
 * until yrss_wait.  Pipeline bursts over several contexts (one per slot). */
#define YRSS_F_ASYNC 0x2u
int yrss_dispatch_burst(yrss_ctx *ctx, void *const *mbufs, uint32_t n,
                        int16_t *out_q, uint32_t *out_hash, uint32_t *out_qidx,
                        uint32_t *out_qstart, uint32_t flags);

/* Zero-copy variant: the mbufs (headers and data) live in host memory that was
 * registered with yrss_register_host_memory (e.g. the DPDK mbuf pool's
 * memzones).  Only the mbuf pointer array crosses PCIe host->device; a gfx950
 * kernel reads each mbuf's buf_addr/data_off/data_len and the header window
 * straight from host memory, and with YRSS_F_WRITE_RSS writes hash.rss back
 * into the mbuf itself.  The dispatcher core does no per-packet work.
 * Returns -EFAULT if a mbuf or its data lies outside every registered range
 * (checked on the GPU; results are then not written).  Synchronous unless
 * flags has YRSS_F_ASYNC. */
int yrss_dispatch_burst_zc(yrss_ctx *ctx, void *const *mbufs, uint32_t n, int16_t *out_q,
                           uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart,
                           uint32_t flags);

/* Zero-copy frames: (data pointer, data_len) pairs the host already holds —
 * e.g. read from the cache-hot mbuf headers right after rte_eth_rx_burst — so
 * the GPU reads only the header windows from registered host memory (one
 * 64-byte PCIe read per packet).  Synchronous.
 *
 * For both zero-copy calls, pointer/length arrays and output arrays that lie
 * in registered memory are read and written in place (no staging copies). */
int yrss_dispatch_frames_zc(yrss_ctx *ctx, const uint8_t *const *data, const uint16_t *len,
                            uint32_t n, int16_t *out_q, uint32_t *out_hash,
                            uint32_t *out_qidx, uint32_t *out_qstart);
/* Same, with flags (YRSS_F_ASYNC). */
int yrss_dispatch_frames_zc_ex(yrss_ctx *ctx, const uint8_t *const *data, const uint16_t *len,
                               uint32_t n, int16_t *out_q, uint32_t *out_hash,
                               uint32_t *out_qidx, uint32_t *out_qstart, uint32_t flags);

/* Complete the burst queued with YRSS_F_ASYNC: 0 (outputs valid), or the error
 * the synchronous call would have returned (-EFAULT, -EIO, ...).  0 when
 * nothing is in flight. */
int yrss_wait(yrss_ctx *ctx);

/* Register / unregister a host range (hipHostRegister, mapped) for the
 * zero-copy path; up to 16 ranges per context.  Unregistering returns -EBUSY
 * while a persistent-worker burst of the context is pending (not yet polled):
 * it may still read mbufs or write outputs in that range. */
#define YRSS_MAX_HOST_RANGES 16
int yrss_register_host_memory(yrss_ctx *ctx, void *base, size_t len);
int yrss_unregister_host_memory(yrss_ctx *ctx, void *base);

/* Same, for frames given as (data pointer, data_len) pairs. */
int yrss_dispatch_frames(yrss_ctx *ctx, const uint8_t *const *data,
                         const uint16_t *len, uint32_t n, int16_t *out_q,
                         uint32_t *out_hash, uint32_t *out_qidx,
                         uint32_t *out_qstart);

/* ---- per-packet registration ------------------------------ */

/* The reference's per-packet hook, unchanged:
 *   typedef int (*dispatch_func_t)(void *data, uint16_t len, uint16_t queue_id,
 *                                  uint16_t nb_queues);            fs/lib/ff_api.h:167
 *   ff_regist_packet_dispatcher(yrss_toeplitz_dispatch);           fs/lib/ff_api.h:170
 * yrss_toeplitz_dispatch has toeplitz_dispatch's signature and return values
 * (fs/lib/ff_dpdk_if.c:1945-2113): the target queue, default_Q (2) for unhashed
 * packets, -1 on error (no context set, a failed GPU call), which F-Stack
 * answers by freeing the mbuf (ff_dpdk_if.c:1080-1083).  queue_id and
 * nb_queues are unused, as in the reference.  dispatch_func_t carries no
 * context, so yrss_set_dispatch_ctx names the one to use (NULL clears it;
 * yrss_fini clears it for its own context).  Every call is a one-packet GPU
 * burst with its own launch and synchronisation (10.8 µs per call measured);
 * if the context has a resident worker (yrss_worker_start), the call is a
 * one-packet worker burst instead, no HIP call (9.3 µs; the window is copied
 * into a slot the context registers on first use; the shim then shares that
 * worker's ring, so submit nothing else to the context while shim calls run:
 * a slot still holding an unpolled ticket makes the call return -1).  A
 * drop-in for registration, not the fast path — use the burst hook or the
 * worker.
 * Calls from several threads (soft_dispatch=0 runs the dispatcher on every
 * lcore, ff_dpdk_if.c:1653) are serialised by one process-wide mutex.  Give the
 * shim a context of its own: while that context has a YRSS_F_ASYNC burst
 * pending the call returns -1, and F-Stack frees the mbuf. */
int yrss_set_dispatch_ctx(yrss_ctx *ctx);
int yrss_toeplitz_dispatch(void *data, uint16_t len, uint16_t queue_id, uint16_t nb_queues);

/* ---- burst routing: process_packets' hand-off --------- */

/* Caller-side plumbing, so the routing drives real DPDK objects:
 *   enqueue  rte_ring_enqueue_burst(dispatch_ring[port][queue], objs, n) —
 *            returns how many of objs (a prefix) were enqueued
 *   clone    pktmbuf_deep_clone(m, pool of queue) (ff_dpdk_if.c:1009-1056);
 *            NULL when the pool is exhausted
 *   release  rte_pktmbuf_free(m) */
struct yrss_route_ops {
    unsigned (*enqueue)(void *user, uint16_t queue, void *const *objs, unsigned n);
    void *(*clone)(void *user, void *mbuf, uint16_t queue);
    void (*release)(void *user, void *mbuf);
    void *user;
};

struct yrss_route_result {
    uint32_t n_local;         /* out_local[]: ff_veth_input on this lcore, in order */
    uint32_t n_kni;           /* out_kni[]: ff_kni_enqueue, in order                */
    uint32_t n_freed;         /* bad queue, ring full or failed clone enqueue       */
    uint32_t n_arp;           /* ARP packets kept local (and cloned)               */
    uint32_t n_unresolved;    /* YRSS_FILTER_TRUNC/LOOP packets, left in out_local */
    uint32_t n_ring[YRSS_MAX_QUEUES];   /* objects enqueued per queue ring        */
};

/* process_packets(port, queue_id, mbufs, n, ctx, pkts_from_ring=0) with the
 * dispatcher registered (ff_dpdk_if.c:1058-1140), for a whole burst: classify
 * on the GPU (queue + protocol_filter), then per packet in order
 *   ret < 0 || ret >= nb_queues        -> release (:1080-1083)
 *   ret != queue_id                    -> ring[ret], FIFO; release if full (:1087-1093)
 *   local, FILTER_ARP                  -> clone to every other queue's ring, a KNI
 *                                         clone if KNI is on and kni_primary, and
 *                                         local input (:1097-1129)
 *   local, KNI accept/reject rule      -> out_kni (:1132-1135)
 *   local, otherwise                   -> out_local (:1137)
 * Ring order equals the reference's one-at-a-time enqueue order.  out_local and
 * out_kni need room for n (+ n ARP clones for out_kni). */
int yrss_route_burst(yrss_ctx *ctx, void *const *mbufs, uint32_t n, uint16_t queue_id,
                     int kni_primary, const struct yrss_route_ops *ops, void **out_local,
                     void **out_kni, struct yrss_route_result *res);

/* ---- connect-side RSS check ----------------------------- */

/* One ff_rss_check call (fs/lib/ff_dpdk_if.c:1904-1940): addresses and ports
 * exactly as the caller stores them (network byte order, in_pcb.c:1155-1156
 * passes faddr, laddr, fport, lport). */
struct yrss_rss_tuple {
    uint32_t saddr;
    uint32_t daddr;
    uint16_t sport;
    uint16_t dport;
};

/* For n tuples in HBM: d_ok[i] = ff_rss_check(...) (1 when nb_queues <= 1, else
 * ((hash & (reta_size - 1)) % nb_queues) == queueid), d_hash[i] (may be NULL)
 * the Toeplitz hash of the 12 raw tuple bytes.  Asynchronous. */
int yrss_rss_check_dev(yrss_ctx *ctx, const struct yrss_rss_tuple *d_tuples, uint32_t n,
                       uint16_t nb_queues, uint16_t reta_size, uint16_t queueid,
                       uint8_t *d_ok, uint32_t *d_hash, void *stream);

/* The whole ephemeral-port search of in_pcbconnect_setup (in_pcb.c:1131-1170)
 * in one launch: bit (p & 31) of bitmap[p >> 5] is ff_rss_check(faddr, laddr,
 * fport, p) for every stored (network-order) lport value p in 0..65535.
 * bitmap is 2048 host words.  Synchronous. */
int yrss_rss_lport_sweep(yrss_ctx *ctx, uint32_t faddr, uint32_t laddr, uint16_t fport,
                         uint16_t nb_queues, uint16_t reta_size, uint16_t queueid,
                         uint32_t *bitmap);

/* ---- multi-GPU sharding ------------------------------------------ */

/* One yrss_ctx and one stream per GPU; each classifies a contiguous shard of the
 * batch with no collective.  yrss_shard_range gives shard `rank` of `world`
 * (balanced: the first n_total % world shards get one packet more).
 * yrss_merge_queue_lists concatenates the shards' per-queue lists in shard
 * order, which keeps every queue FIFO over the whole batch, as the reference's
 * rte_ring does (fs/lib/ff_dpdk_if.c:1087-1093): nbk = nb_queues + 1 buckets;
 * shard s holds qidx[s] (shard-local indices) and qstart[s] (nbk + 1 offsets)
 * and starts at global packet first[s]; out_qidx gets global indices (64-bit:
 * a node's batch can exceed 2^32 packets), out_qstart nbk + 1 offsets.
 * Host-only.  yastack_amd/shard.py is the Python twin. */
int yrss_shard_range(uint64_t n_total, uint32_t world, uint32_t rank, uint64_t *first,
                     uint64_t *count);
int yrss_merge_queue_lists(uint32_t nshards, uint32_t nbk, const uint64_t *first,
                           const uint32_t *const *qidx, const uint32_t *const *qstart,
                           uint64_t *out_qidx, uint64_t *out_qstart);

/* ---- pcap capture I/O ----------------------------------- */

/* ff_enable_pcap + ff_dump_packets (fs/lib/ff_dpdk_pcap.c:49-102) for a burst:
 * append == 0 creates the file with the reference's 24-byte header (magic
 * 0xA1B2C3D4, v2.4, snaplen 65535, LINKTYPE_ETHERNET); every frame gets a
 * 16-byte record {sec, usec, caplen = len, len} and its bytes.  ts_* may be
 * NULL (zeros).  Host file I/O only. */
int yrss_pcap_write(const char *path, int append, const uint8_t *const *data,
                    const uint32_t *len, uint32_t n, const uint32_t *ts_sec,
                    const uint32_t *ts_usec);

/* Replay: records [first, first+max) of an Ethernet pcap (either byte order,
 * usec or nsec magic) into header windows of `stride` bytes (>= 64) plus
 * data_len = min(caplen, 65535) — each record is one single-segment mbuf —
 * and, if non-NULL, the wire length.  Returns the number of records read, or
 * -errno.  max == 0 returns the capture's record count. */
int yrss_pcap_read(const char *path, uint64_t first, uint32_t max, uint8_t *win,
                   uint32_t stride, uint16_t *len, uint32_t *wire_len);

/* ---- synthetic traffic (bench / parity inputs; see yrss_synth.h) ------------- */

struct yrss_synth_params;
/* Write header windows + data_len of packets [first, first+n) of a synthetic
 * stream directly into HBM.  Bit-identical to yrss_synth_window() on the host. */
int yrss_synth_dev(yrss_ctx *ctx, const struct yrss_synth_params *p,
                   uint64_t first, uint32_t n, uint8_t *d_win,
                   uint32_t win_stride, uint16_t *d_len, void *stream);

/* ---- timing hook (bench) ------------------------------------------------------- */

/* kernel_mask bit k (YRSS_K_*) brackets every launch of kernel k by
 * yrss_dispatch_dev with hipEvents on the launch stream (0 disables; enabling
 * resets the totals).  yrss_timing_read synchronises the pending events and
 * returns the summed milliseconds and launch count for one kernel. */
#define YRSS_K_PARSE_HASH 0
#define YRSS_K_SCAN       1
#define YRSS_K_SCATTER    2
#define YRSS_K_COUNT      3
/* Kernel ids that appear only in fault records (not timed). */
#define YRSS_K_BURST      8   /* yrss_burst_small: one-launch bursts / batches */
#define YRSS_K_WORKER     9   /* yrss_burst_worker */
int yrss_timing_enable(yrss_ctx *ctx, int kernel_mask);
int yrss_timing_read(yrss_ctx *ctx, int kernel, double *total_ms,
                     uint32_t *launches);
/* The q-quantile (0.5: median) of kernel k's per-launch
 * durations since yrss_timing_enable, in ms; -ENODATA before any launch. */
int yrss_timing_quantile(yrss_ctx *ctx, int kernel, double q, double *ms);

/* ---- persistent burst worker ------------------------------------------------------ */

/* Small bursts with no kernel launch and no stream synchronisation per burst:
 * a persistent gfx950 kernel (nblocks workgroups, one CU each) polls a ring of
 * nslots slots in host-coherent pinned memory.  Submit copies the mbuf pointer
 * array into a slot and publishes it; the kernel reads the mbufs (which must
 * lie in memory registered with yrss_register_host_memory) over PCIe and
 * classifies them like yrss_dispatch_burst_zc.  Output arrays that lie in
 * registered memory are written in place; others are written into the slot
 * and copied to the caller's arrays by the poll.  Up to nslots bursts are in
 * flight; every ticket must be polled before its slot is reused (submit
 * returns -EBUSY otherwise).  The kernel leaves after YRSS_WORKER_IDLE_MS
 * (default 50) without a submit or YRSS_WORKER_LIFE_MS (default 1000) in total
 * and is relaunched transparently by the next submit or poll (also by a
 * wait = 0 poll); registering or unregistering host memory restarts it.
 * nslots is a multiple of nblocks; nb_queues + 1 <= 64.  Submits and polls of
 * one context come from one thread at a time (the dispatcher lcore). */
#define YRSS_WORKER_MAX_BURST 1024
#define YRSS_WORKER_MAX_BLOCKS 128
#define YRSS_WORKER_MAX_SLOTS 4096
int yrss_worker_start(yrss_ctx *ctx, uint32_t nslots, uint32_t nblocks);
/* Queue one burst (n <= YRSS_WORKER_MAX_BURST; flags: YRSS_F_WRITE_RSS);
 * *ticket identifies it for yrss_worker_poll.  The output arrays must stay
 * valid until the ticket is polled. */
int yrss_worker_submit(yrss_ctx *ctx, void *const *mbufs, uint32_t n, int16_t *out_q,
                       uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart,
                       uint32_t flags, uint64_t *ticket);
/* Same for (data pointer, data_len) pairs the host already holds, like
 * yrss_dispatch_frames_zc: the GPU reads only the windows (in registered
 * memory). */
int yrss_worker_submit_frames(yrss_ctx *ctx, const uint8_t *const *data, const uint16_t *len,
                              uint32_t n, int16_t *out_q, uint32_t *out_hash,
                              uint32_t *out_qidx, uint32_t *out_qstart, uint64_t *ticket);
/* Same for windows the caller has copied, contiguously, into registered
 * memory: window i at win + i * stride holds the first min(len[i], stride)
 * bytes of packet i's first segment (stride >= 64, a multiple of 16; 80 never
 * truncates).  The GPU reads the burst as one stretch of host memory, with no
 * per-packet pointer reads: the dispatcher lcore's copy of each window (cache
 * hot after rte_eth_rx_burst) replaces the GPU's dependent PCIe reads of the
 * pointer array and then each scattered window.  -EFAULT if the windows are
 * not in registered memory. */
int yrss_worker_submit_windows(yrss_ctx *ctx, const uint8_t *win, uint32_t stride,
                               const uint16_t *len, uint32_t n, int16_t *out_q,
                               uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart,
                               uint64_t *ticket);
/* 0: the burst is done and its outputs in place; -EAGAIN: not yet (wait = 0);
 * -EFAULT: a mbuf or its data lies outside every registered range;
 * -ETIMEDOUT: waited 10 s (a burst takes microseconds: the GPU is hung).  The
 * context is then marked hung: yrss_fini neither waits for the device nor
 * frees memory a still-running kernel may write (it is left to process exit). */
int yrss_worker_poll(yrss_ctx *ctx, uint64_t ticket, int wait);
/* Stop the kernel and free the ring (also done by yrss_fini). */
int yrss_worker_stop(yrss_ctx *ctx);

/* ---- host bursts fanned out over several GPUs ------------------- */

/* The reference's soft dispatch is ONE lcore feeding every dispatch ring
 * (fs/lib/ff_dpdk_if.c:1653-1683).  A fan-out keeps that single dispatcher
 * thread and spreads its consecutive bursts round-robin over nctx contexts,
 * each with its own persistent worker (yrss_worker_*) on its own device and
 * PCIe link: burst g (tickets 1, 2, ...) goes to context (g - 1) % nctx.
 * yrss_fanout_next returns tickets in submission order as they complete, so
 * handing each burst's per-queue lists to the rings in that order keeps every
 * queue FIFO over the whole stream, as rte_ring does (:1087-1093).  devices may
 * repeat (several contexts on one GPU).  Host memory is registered with every
 * context.  Submit and next come from one thread (the dispatcher lcore); each
 * context holds up to nslots bursts, and a ticket must be returned by
 * yrss_fanout_next before its context's slot is reused (submit: -EBUSY). */
#define YRSS_FANOUT_MAX_CTX 64
typedef struct yrss_fanout yrss_fanout;
int yrss_fanout_init(const struct yrss_config *cfg, const int *devices, uint32_t nctx,
                     uint32_t nslots, uint32_t nblocks, yrss_fanout **out);
int yrss_fanout_fini(yrss_fanout *f);
uint32_t yrss_fanout_size(yrss_fanout *f);
int yrss_fanout_register_host_memory(yrss_fanout *f, void *base, size_t len);
int yrss_fanout_unregister_host_memory(yrss_fanout *f, void *base);
/* As yrss_worker_submit / yrss_worker_submit_frames; *ticket is the fan-out's. */
int yrss_fanout_submit(yrss_fanout *f, void *const *mbufs, uint32_t n, int16_t *out_q,
                       uint32_t *out_hash, uint32_t *out_qidx, uint32_t *out_qstart,
                       uint32_t flags, uint64_t *ticket);
int yrss_fanout_submit_frames(yrss_fanout *f, const uint8_t *const *data, const uint16_t *len,
                              uint32_t n, int16_t *out_q, uint32_t *out_hash,
                              uint32_t *out_qidx, uint32_t *out_qstart, uint64_t *ticket);
/* The oldest ticket not yet returned, once its burst is done: 0 with *ticket
 * set (-EFAULT also sets it: the burst is consumed, a pointer was outside every
 * registered range); -EAGAIN: still running (wait = 0); -ENOENT: nothing
 * outstanding; other errors as yrss_worker_poll. */
int yrss_fanout_next(yrss_fanout *f, int wait, uint64_t *ticket);
/* Host-only: the context serving fan-out ticket `ticket`, and its ticket there. */
int yrss_fanout_route(uint64_t ticket, uint32_t nctx, uint32_t *ctx, uint64_t *ctx_ticket);

/* ---- device-side status ----------------------------------------------------------- */

/* Every index the per-queue lists are built from (count slots, stage slots,
 * list slots) is bounds-checked on the GPU.  A check that fails stores nothing
 * and sets the context's fault record (first fault wins): that batch's
 * qidx/qstart are invalid; q and hash are not affected.  Codes: */
#define YRSS_FAULT_NONE           0
#define YRSS_FAULT_SCAN_TIMEOUT   1   /* scan look-back did not resolve: where = bucket row  */
#define YRSS_FAULT_LIST_RANGE     2   /* list slot >= n: where = packet, value = slot        */
#define YRSS_FAULT_COUNT_MISMATCH 3   /* a span's histogram differs from the parse counts:
                                         where = span, value = bucket                        */
#define YRSS_FAULT_COUNT_SLOT     4   /* parse count slot beyond LDS: where = wave, value = slot */
#define YRSS_FAULT_STAGE          5   /* scatter stage slot out of range: where = packet     */
#define YRSS_FAULT_LINE_CAPACITY  6   /* a line-scatter kernel launched for more buckets than
                                         its per-bucket arrays hold (the host refuses such a
                                         plan with -EINVAL; the kernel checks again at entry
                                         and leaves): where = buckets, value = its capacity */
struct yrss_fault {
    uint32_t code;     /* YRSS_FAULT_*                                   */
    uint32_t kernel;   /* YRSS_K_* of the kernel whose guard fired       */
    uint32_t where;
    uint32_t value;
};

/* Synchronises the context's own streams (its internal one and the stream of
 * its last device batch, not the whole device) and reports (then clears) the
 * fault record: 0 = no guard fired since the last call, -EIO = one did (the
 * record is printed to stderr).  The host-synchronous entry points check it
 * themselves and return -EIO.  A persistent-worker burst carries its own
 * record: yrss_worker_poll returns -EIO for exactly the burst whose guard
 * fired (other bursts in flight are unaffected) and copies the record here
 * when this one is empty.  The reference has no equivalent: its per-packet
 * rte_ring_enqueue cannot fail this way (ff_dpdk_if.c:1087-1093). */
int yrss_status(yrss_ctx *ctx);
/* Same, copying the record (code 0 = none) instead of printing it. */
int yrss_fault_info(yrss_ctx *ctx, struct yrss_fault *out);

/* ---- layout overrides (tests and measurements) ------------------------------------ */

/* Every field 0 (scatter_xcd -1) is the built-in default; results never
 * depend on these, only the work layout does. */
struct yrss_tuning {
    uint32_t chunk_tiles;    /* parse chunk in 64-packet tiles, power of two (default 4
                                up to 16 buckets, 8 to 128, 16 beyond; larger when a
                                wave's count slots run out)                          */
    uint32_t span_tiles;     /* line-scatter span in tiles, power of two (default 128
                                up to 128 buckets, 256 beyond)                       */
    uint32_t parse_blocks;   /* parse grid (default one workgroup per CU)            */
    uint32_t one_launch;     /* batches <= 4096 packets in one launch: 0 host bursts
                                and device batches, 1 host bursts only, 2 never      */
    int32_t  scatter_xcd;    /* XCD-contiguous scatter ranges: -1 default (on), 0, 1 */
    uint32_t scan_kernel;    /* per-chunk list prefixes: 0 default (up to 16 buckets
                                inside the line scatter, no scan kernel), 1 always
                                the scan kernel                                      */
};
int yrss_set_tuning(yrss_ctx *ctx, const struct yrss_tuning *t);

/* ---- introspection --------------------------------------------------------------- */

const char *yrss_version(void);
/* Kernel-name string as it appears in rocprof traces, for kernel id k. */
const char *yrss_kernel_name(int kernel);
/* Number of workgroups the parse+hash kernel will use for n packets. */
uint32_t yrss_grid_for(yrss_ctx *ctx, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif /* YRSS_H */
