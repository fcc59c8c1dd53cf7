/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A clean-room CPU restatement of yastack's soft-RSS path, written from the
 * behaviour specified in SURVEY.md §8(a) and checked line by line against the
 * reference source.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker or the
 * timed CPU baseline — never as part of the product path (yastack_amd/ and
 * include/ do not link it; the product fails loudly without its HIP library).
 *
 * Parity pinning:
 *   - Toeplitz engine: Intel 82599 verification vectors held by the
 *     reference's own test (dpdk/test/test/test_thash.c:60-104), and the
 *     reference's toeplitz_hash compiled from its source into oracle/_ref by
 *     oracle/build_ref.sh (random-input cross-check).
 *   - Dispatch (byte order, length checks, queue mapping): the known-answer
 *     table produced by running the reference toeplitz_dispatch in the survey
 *     container (committed as tests/golden/survey_kat.json).
 *
 * Reference functions restated here (yastack tree, read-only):
 *   toeplitz_hash        fs/lib/ff_dpdk_if.c:1881-1902
 *   toeplitz_dispatch    fs/lib/ff_dpdk_if.c:1945-2113
 *   process_packets      fs/lib/ff_dpdk_if.c:1058-1094 (dispatcher block)
 *   ff_rss_check         fs/lib/ff_dpdk_if.c:1904-1940
 *   protocol_filter      fs/lib/ff_dpdk_if.c:976-996, ff_dpdk_kni.c:218-290
 *   kni_set_bitmap       fs/lib/ff_dpdk_kni.c:84-118
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/yrss_synth.h"

#define YRSS_ORACLE_MAXB 258   /* YRSS_MAX_QUEUES + drop bucket + 1 */

struct oracle_cfg {
    uint8_t  key[40];
    uint32_t keylen;
    int32_t  nb_procs;
    uint16_t nb_queues;
    uint8_t  soft_dispatch;
    uint8_t  dispatch_only_core;
};

/* ---- Toeplitz engine ------------------------------------------------------- */

/* Bit-serial Toeplitz, ff_dpdk_if.c:1881-1902.  A 32-bit window slides over
 * the key, one key bit per input bit, MSB first; every set input bit XORs the
 * current window into the result.  Key bits past keylen shift in as zero. */
uint32_t oracle_toeplitz_hash(unsigned keylen, const uint8_t *key,
                              unsigned datalen, const uint8_t *data)
{
    uint32_t win = ((uint32_t)key[0] << 24) | ((uint32_t)key[1] << 16) |
                   ((uint32_t)key[2] << 8) | (uint32_t)key[3];
    uint32_t acc = 0;
    for (unsigned byte = 0; byte < datalen; ++byte) {
        const unsigned next_key = byte + 4;          /* key byte feeding the window */
        for (unsigned bit = 0; bit < 8; ++bit) {
            const unsigned mask = 0x80u >> bit;
            if (data[byte] & mask)
                acc ^= win;
            win <<= 1;
            if (next_key < keylen && (key[next_key] & mask))
                win |= 1u;
        }
    }
    return acc;
}

/* Equivalent byte-table formulation: T[j][v] = XOR of the key windows at bit
 * positions 8j+b for every set bit b of v (MSB first).  Used by the fast CPU
 * baseline; identical output to oracle_toeplitz_hash for datalen <= 12. */
void oracle_build_tables(unsigned keylen, const uint8_t *key, uint32_t tbl[12][256])
{
    uint32_t kwin[96];
    for (unsigned k = 0; k < 96; ++k) {
        uint32_t w = 0;
        for (unsigned b = 0; b < 32; ++b) {
            const unsigned bit = k + b, kb = bit >> 3;
            const unsigned v = (kb < keylen) ? (key[kb] >> (7 - (bit & 7))) & 1u : 0u;
            w = (w << 1) | v;
        }
        kwin[k] = w;
    }
    for (unsigned j = 0; j < 12; ++j)
        for (unsigned v = 0; v < 256; ++v) {
            uint32_t acc = 0;
            for (unsigned b = 0; b < 8; ++b)
                if (v & (0x80u >> b))
                    acc ^= kwin[8 * j + b];
            tbl[j][v] = acc;
        }
}

static uint32_t hash_tables(const uint32_t tbl[12][256], const uint8_t t[12])
{
    uint32_t h = 0;
    for (int j = 0; j < 12; ++j)
        h ^= tbl[j][t[j]];
    return h;
}

/* ---- toeplitz_dispatch ------------------------------------------------------- */

/* Restatement of toeplitz_dispatch (ff_dpdk_if.c:1945-2113).  Returns the
 * queue; hashed and hash report whether the Toeplitz hash was computed.
 * tbl == NULL selects the bit-serial engine. */
static int dispatch_one(const uint8_t *b, uint16_t len, const struct oracle_cfg *c,
                        const uint32_t (*tbl)[256], uint32_t *hash, int *hashed)
{
    *hash = 0;
    *hashed = 0;
    if (len < 14)                                  /* :1956-1957 ETHER_HDR_LEN */
        return 2;
    const unsigned et = ((unsigned)b[12] << 8) | b[13];   /* ntohs(ether_type) */
    switch (et) {
    case 0x0800: {                                 /* ETHER_TYPE_IPv4 :1964   */
        const uint16_t ip_len = (uint16_t)(len - 14);
        if (ip_len < 20)                           /* sizeof(ipv4_hdr) :1968  */
            return 2;
        const int ihl4 = (b[14] & 0x0f) << 2;      /* version nibble unchecked */
        if (ip_len < ihl4)                         /* :1974-1976              */
            return 2;
        const uint16_t pay_len = (uint16_t)(len - ihl4);  /* NB: not minus 14 */
        if (pay_len < 20)                          /* sizeof(tcp_hdr) :1981   */
            return 2;
        if (b[23] != 6)                            /* UDP, IPIP, others → 2   */
            return 2;
        /* IPPROTO_TCP: len < 20 cannot hold here (len >= 34).  The tuple is the
         * little-endian memory image of ntohl(src), ntohl(dst), ntohs(sport),
         * ntohs(dport) copied with bcopy (:1994-2021): each field's bytes are
         * reversed relative to the wire. */
        const int p = 14 + ihl4;
        uint8_t t[12];
        t[0] = b[29]; t[1] = b[28]; t[2] = b[27]; t[3] = b[26];
        t[4] = b[33]; t[5] = b[32]; t[6] = b[31]; t[7] = b[30];
        t[8] = b[p + 1]; t[9] = b[p]; t[10] = b[p + 3]; t[11] = b[p + 2];
        const uint32_t h = tbl ? hash_tables(tbl, t)
                               : oracle_toeplitz_hash(c->keylen, c->key, 12, t);
        *hash = h;
        *hashed = 1;
        uint16_t q;                                /* uint16_t default_Q       */
        if (c->soft_dispatch && c->dispatch_only_core)   /* :2031-2032 */
            q = (uint16_t)(h % (unsigned)(c->nb_procs - 1) + 1u);
        else                                             /* :2034 */
            q = (uint16_t)(h % (unsigned)c->nb_procs);
        return q;
    }
    case 0x0806:                                   /* ETHER_TYPE_ARP  :2063 */
    case 0x8035:                                   /* ETHER_TYPE_RARP :2068 */
        return 0;
    default:                                       /* IPv6, VLAN, QinQ, ... */
        return 2;
    }
}

int oracle_toeplitz_dispatch(const uint8_t *data, uint16_t len,
                             const struct oracle_cfg *c, uint32_t *hash_out)
{
    uint32_t h;
    int hashed;
    const int q = dispatch_one(data, len, c, NULL, &h, &hashed);
    if (hash_out)
        *hash_out = h;
    return q;
}

/* Batch over header windows (the yrss_dispatch_dev input layout).  Adds the
 * boundary's one rule the reference cannot have: a hashed packet whose ports
 * end beyond the staged window (18 + 4*IHL > stride) is YRSS_Q_TRUNCATED. */
void oracle_dispatch_windows(const uint8_t *win, uint32_t stride, const uint16_t *len,
                             uint32_t n, const struct oracle_cfg *c, int16_t *q,
                             uint32_t *hash, int fast)
{
    static uint32_t tbl[12][256];
    if (fast)
        oracle_build_tables(c->keylen, c->key, tbl);
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t *b = win + (size_t)i * stride;
        uint32_t h;
        int hashed;
        int r = dispatch_one(b, len[i], c, fast ? (const uint32_t(*)[256])tbl : NULL,
                             &h, &hashed);
        if (hashed && 18u + 4u * (b[14] & 0x0fu) > stride) {
            r = -2;
            h = 0;
        }
        q[i] = (int16_t)r;
        if (hash)
            hash[i] = h;
    }
}

/* ---- process_packets dispatcher block ----------------------------------------- */

/* Per-queue FIFO lists, ff_dpdk_if.c:1078-1094: ret < 0 || ret >= nb_queues is
 * freed (bucket nb_queues); otherwise the mbuf goes to dispatch_ring[port][ret]
 * (rte_ring is FIFO, so packet order is kept inside each queue). */
void oracle_process_burst(const int16_t *q, uint32_t n, uint16_t nb_queues,
                          uint32_t *qidx, uint32_t *qstart)
{
    const uint32_t nb = (uint32_t)nb_queues + 1u;
    for (uint32_t b = 0; b <= nb; ++b)
        qstart[b] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const int r = q[i];
        const uint32_t b = (r >= 0 && r < (int)nb_queues) ? (uint32_t)r : nb_queues;
        qstart[b + 1]++;
    }
    for (uint32_t b = 0; b < nb; ++b)
        qstart[b + 1] += qstart[b];
    /* stable placement: walk packets in order */
    uint32_t fill[YRSS_ORACLE_MAXB];
    for (uint32_t b = 0; b < nb; ++b)
        fill[b] = qstart[b];
    for (uint32_t i = 0; i < n; ++i) {
        const int r = q[i];
        const uint32_t b = (r >= 0 && r < (int)nb_queues) ? (uint32_t)r : nb_queues;
        qidx[fill[b]++] = i;
    }
}

/* ---- ff_rss_check ------------------------------------------ */

/* ff_dpdk_if.c:1904-1940: tuple = raw (network-order) saddr, daddr, sport,
 * dport as stored in the caller's variables; RETA-masked modulo. */
int oracle_ff_rss_check(const struct oracle_cfg *c, uint16_t nb_queues,
                        uint16_t reta_size, uint16_t queueid, uint32_t saddr,
                        uint32_t daddr, uint16_t sport, uint16_t dport)
{
    if (nb_queues <= 1)
        return 1;
    uint8_t t[12];
    memcpy(t, &saddr, 4);
    memcpy(t + 4, &daddr, 4);
    memcpy(t + 8, &sport, 2);
    memcpy(t + 10, &dport, 2);
    const uint32_t h = oracle_toeplitz_hash(c->keylen, c->key, 12, t);
    return ((h & (uint32_t)(reta_size - 1)) % nb_queues) == queueid;
}

/* ---- synthetic input + timing helpers ------------------------------------------ */

void oracle_synth(const struct yrss_synth_params *p, uint64_t first, uint32_t n,
                  uint8_t *win, uint32_t stride, uint16_t *len)
{
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t w[20];
        yrss_synth_window(p, first + i, w, &len[i]);
        uint8_t *dst = win + (size_t)i * stride;
        const uint32_t nb = stride < 80 ? stride : 80;
        for (uint32_t k = 0; k < nb; ++k)
            dst[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
        for (uint32_t k = nb; k < stride; ++k)
            dst[k] = (uint8_t)(k * 131u + (uint32_t)i);
    }
}

/* CPU-baseline loop: `reps` passes of the dispatcher over the sample, one call
 * per packet exactly as process_packets does.  Returns a checksum so the work
 * cannot be elided. */
uint64_t oracle_bench_dispatch(const uint8_t *win, uint32_t stride, const uint16_t *len,
                               uint32_t n, const struct oracle_cfg *c, uint32_t reps,
                               int fast)
{
    static uint32_t tbl[12][256];
    if (fast)
        oracle_build_tables(c->keylen, c->key, tbl);
    uint64_t sum = 0;
    for (uint32_t r = 0; r < reps; ++r)
        for (uint32_t i = 0; i < n; ++i) {
            uint32_t h;
            int hashed;
            const int q = dispatch_one(win + (size_t)i * stride, len[i], c,
                                       fast ? (const uint32_t(*)[256])tbl : NULL, &h,
                                       &hashed);
            sum += (uint64_t)q * 0x9E3779B97F4A7C15ull + h;
        }
    return sum;
}

/* The reference calls its dispatcher through a function pointer registered
 * with ff_regist_packet_dispatcher: `int ret = (*packet_dispatcher)(data, len,
 * queue_id, nb_queues)` (ff_dpdk_if.c:1078-1079, dispatch_func_t at
 * ff_api.h:167-168), and toeplitz_dispatch reads its knobs from the global
 * ff_global_cfg.  These wrappers have that signature and read a file-scope
 * config; g_dispatcher is volatile so the compiler cannot inline the call. */
static const struct oracle_cfg *g_cfg;
static uint32_t g_tbl[12][256];

static int dispatcher_bit_serial(void *data, uint16_t len, uint16_t queue_id, uint16_t nb_queues)
{
    uint32_t h;
    int hashed;
    (void)queue_id;
    (void)nb_queues;
    return dispatch_one((const uint8_t *)data, len, g_cfg, NULL, &h, &hashed);
}

static int dispatcher_table(void *data, uint16_t len, uint16_t queue_id, uint16_t nb_queues)
{
    uint32_t h;
    int hashed;
    (void)queue_id;
    (void)nb_queues;
    return dispatch_one((const uint8_t *)data, len, g_cfg, (const uint32_t(*)[256])g_tbl, &h,
                        &hashed);
}

typedef int (*oracle_dispatch_fn)(void *data, uint16_t len, uint16_t queue_id, uint16_t nb_queues);
static oracle_dispatch_fn volatile g_dispatcher;

static uint64_t mono_ns(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

/* CPU-baseline window with a wall-clock deadline, so that every process of a
 * multi-core cell runs over the same stretch of time: spin until start_ns
 * (CLOCK_MONOTONIC), then pass over the sample packet by packet until end_ns
 * (checked every 4096 packets).  call = 0: dispatch_one inlined, as
 * oracle_bench_dispatch; call = 1: through the registered-dispatcher function
 * pointer, as process_packets calls it.  out = {packets, first ns, last ns}.
 * Returns a checksum so the work cannot be elided. */
uint64_t oracle_bench_window(const uint8_t *win, uint32_t stride, const uint16_t *len,
                             uint32_t n, const struct oracle_cfg *c, int fast, int call,
                             uint64_t start_ns, uint64_t end_ns, uint64_t out[3])
{
    static uint32_t tbl[12][256];
    if (fast) {
        oracle_build_tables(c->keylen, c->key, tbl);
        memcpy(g_tbl, tbl, sizeof(tbl));
    }
    g_cfg = c;
    g_dispatcher = fast ? dispatcher_table : dispatcher_bit_serial;
    /* sleep, not spin, until the common start: spinning processes use up a
     * cgroup CPU quota before the window opens, and the throttled ones then
     * start late (round 5's first 16-core cells overlapped 0.69) */
    const struct timespec ts = {(time_t)(start_ns / 1000000000ull), (long)(start_ns % 1000000000ull)};
    while (clock_nanosleep(CLOCK_MONOTONIC, TIMER_ABSTIME, &ts, NULL) != 0)
        ;
    while (mono_ns() < start_ns)
        ;
    const uint64_t t0 = mono_ns();
    uint64_t sum = 0, done = 0, t1 = t0;
    uint32_t i = 0;
    for (;;) {
        const uint32_t e = i + 4096u < n ? i + 4096u : n;
        done += e - i;
        if (call) {
            for (; i < e; ++i) {
                const int q = g_dispatcher((void *)(win + (size_t)i * stride), len[i], 0,
                                           (uint16_t)c->nb_queues);
                sum += (uint64_t)q * 0x9E3779B97F4A7C15ull;
            }
        } else {
            for (; i < e; ++i) {
                uint32_t h;
                int hashed;
                const int q = dispatch_one(win + (size_t)i * stride, len[i], c,
                                           fast ? (const uint32_t(*)[256])tbl : NULL, &h,
                                           &hashed);
                sum += (uint64_t)q * 0x9E3779B97F4A7C15ull + h;
            }
        }
        if (i == n)
            i = 0;
        t1 = mono_ns();
        if (t1 >= end_ns)
            break;
    }
    out[0] = done;
    out[1] = t0;
    out[2] = t1;
    return sum;
}

/* ---- protocol_filter / KNI ---------------------------------- */

/* kni_set_bitmap (ff_dpdk_kni.c:99-118) with set_bitmap (:84-89): a '-' found
 * before the next ',' (at least one char between) makes an atoi range; each
 * value is truncated to uint16_t and stored at bit 0x80 >> (p % 8) of byte
 * p / 8 where p = htons(port). */
static void set_port(uint8_t *bm, uint16_t port)
{
    const uint16_t p = (uint16_t)((port >> 8) | (port << 8));
    bm[p / 8] |= (uint8_t)(0x80 >> (p % 8));
}

void oracle_kni_set_bitmap(const char *s, uint8_t *bm)
{
    if (!s)
        return;
    const char *head = s;
    for (;;) {
        const char *comma = strstr(head, ",");
        const char *dash = strstr(head, "-");
        if (dash && (!comma || dash < comma - 1)) {
            long count = 0;
            for (long v = atol(head); v <= atol(dash + 1) && count < 65536; ++v, ++count)
                set_port(bm, (uint16_t)v);
        } else {
            set_port(bm, (uint16_t)atol(head));
        }
        if (!comma)
            break;
        head = comma + 1;
    }
}

static int port_in(const uint8_t *bm, uint16_t raw)
{
    return (bm[raw / 8] & (0x80 >> (raw % 8))) != 0;
}

/* protocol_filter (ff_dpdk_if.c:976-996) + ff_kni_proto_filter /
 * protocol_filter_ip/_tcp/_udp (ff_dpdk_kni.c:218-290).  `avail` is how many
 * bytes of the frame are readable (the staged window); a header walk that
 * needs more returns -2 (TRUNC).  IHL=0 under IPIP makes the reference recurse
 * on the same header forever: returned as -3 (LOOP) instead of hanging. */
int oracle_protocol_filter(const uint8_t *b, uint16_t len, uint32_t avail, int enable_kni,
                           const uint8_t *tcp_bm, const uint8_t *udp_bm)
{
    if (len < 14)
        return -1;                                    /* FILTER_UNKNOWN */
    const unsigned et = ((unsigned)b[12] << 8) | b[13];
    if (et == 0x0806)
        return 1;                                     /* FILTER_ARP */
    if (!enable_kni || et != 0x0800)
        return -1;
    uint32_t o = 14, left = (uint16_t)(len - 14);
    for (;;) {                                        /* protocol_filter_ip */
        if (left < 20)
            return -1;
        if (o >= avail)
            return -2;
        const uint32_t hl = (b[o] & 0x0f) << 2;
        if (left < hl)
            return -1;
        if (o + 9 >= avail)
            return -2;
        const unsigned pr = b[o + 9];
        const uint32_t nx = o + hl;
        const uint16_t nl = (uint16_t)(left - hl);
        if (pr == 6 || pr == 17) {                    /* _tcp: len>=20, _udp: len>=8 */
            if (nl < (pr == 6 ? 20 : 8))
                return -1;
            if (nx + 3 >= avail)
                return -2;
            const uint16_t raw = (uint16_t)(b[nx + 2] | (b[nx + 3] << 8));  /* hdr->dst_port */
            return port_in(pr == 6 ? tcp_bm : udp_bm, raw) ? 2 : -1;
        }
        if (pr != 4)                                  /* IPPROTO_IPIP recurses */
            return -1;
        if (hl == 0)
            return -3;
        o = nx;
        left = nl;
    }
}

void oracle_filter_windows(const uint8_t *win, uint32_t stride, const uint16_t *len, uint32_t n,
                           int enable_kni, const uint8_t *tcp_bm, const uint8_t *udp_bm,
                           int8_t *out)
{
    for (uint32_t i = 0; i < n; ++i)
        out[i] = (int8_t)oracle_protocol_filter(win + (size_t)i * stride, len[i], stride,
                                                enable_kni, tcp_bm, udp_bm);
}

/* Batch of ff_rss_check calls over raw 12-byte tuples (struct yrss_rss_tuple). */
void oracle_rss_check_batch(const struct oracle_cfg *c, const uint8_t *tuples, uint32_t n,
                            uint16_t nb_queues, uint16_t reta_size, uint16_t queueid,
                            uint8_t *ok, uint32_t *hash)
{
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t s, d;
        uint16_t sp, dp;
        memcpy(&s, tuples + 12 * i, 4);
        memcpy(&d, tuples + 12 * i + 4, 4);
        memcpy(&sp, tuples + 12 * i + 8, 2);
        memcpy(&dp, tuples + 12 * i + 10, 2);
        ok[i] = (uint8_t)oracle_ff_rss_check(c, nb_queues, reta_size, queueid, s, d, sp, dp);
        if (hash)
            hash[i] = oracle_toeplitz_hash(c->keylen, c->key, 12, tuples + 12 * i);
    }
}

/* timing twin of oracle/_ref's ref_bench_hash (CPU-baseline calibration) */
uint32_t oracle_bench_hash(const uint8_t *key, const uint8_t *tuples, unsigned n, unsigned reps)
{
    uint32_t acc = 0;
    for (unsigned r = 0; r < reps; ++r)
        for (unsigned i = 0; i < n; ++i)
            acc += oracle_toeplitz_hash(40, key, 12, tuples + 12 * i);
    return acc;
}
