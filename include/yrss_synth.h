/*
 * yrss_synth.h — deterministic synthetic packet streams for the five
 * BASELINE.json configurations (plus a TCP/IPv4 variant and an adversarial
 * "fuzz" stream for parity).  Header-only, host + device: the same inline
 * function fills windows in HBM (yrss_synth_dev) and in host memory (tests,
 * oracle), so GPU and CPU see bit-identical input.
 *
 * The generator is counter-based (packet i depends only on (seed, i)), so any
 * shard [first, first+n) of a stream can be produced independently on any
 * rank — which is what lets bench.py shard bursts across GPUs without moving
 * data.  It is the build's own traffic model, not code from the reference;
 * frame layouts follow rte_ether.h:298-307 / rte_ip.h:31-42 / rte_tcp.h:26-36
 * of the reference's DPDK 18.02.
 *
 * A window is 80 bytes (YRSS_WIN_FULL) returned as 20 little-endian words:
 * byte k of the frame is (w[k/4] >> (8*(k%4))) & 0xff.  Bytes of a window
 * beyond the frame's data_len are filler the parse never reads.
 */
#ifndef YRSS_SYNTH_H
#define YRSS_SYNTH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define YRSS_SYN_FN static inline __host__ __device__
#else
#define YRSS_SYN_FN static inline
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* Profiles.  Numbers in brackets are BASELINE.json configs[] indices + 1. */
#define YRSS_SYN_UDP4_1FLOW 0 /* [1] 64B Eth/IPv4/UDP, one flow 10.0.0.1:1234->10.0.0.2:5678 */
#define YRSS_SYN_UDP4       1 /* [2] 64B Eth/IPv4/UDP, nflows random 5-tuples               */
#define YRSS_SYN_IMIX       2 /* [3] IMIX 64/570/1500 (7:4:1), TCP:UDP 1:1 per flow         */
#define YRSS_SYN_VLAN6_TCP  3 /* [4] 64B Eth/VLAN/IPv6/TCP                                  */
#define YRSS_SYN_JUMBO_TCP4 4 /* [5] 9000B TCP/IPv4; data_len = first segment = 2048       */
#define YRSS_SYN_TCP4       5 /*     64B Eth/IPv4/TCP (every packet takes the hash path)   */
#define YRSS_SYN_FUZZ       6 /*     adversarial: random ethertype/IHL/proto/len            */
#define YRSS_SYN_NPROFILES  7

struct yrss_synth_params {
    uint64_t seed;
    uint32_t profile;
    uint32_t nflows;   /* >= 1; ignored by UDP4_1FLOW and FUZZ */
};

YRSS_SYN_FN uint64_t yrss_mix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

/* Two bytes of a big-endian u16 placed at byte offset o (0..2) of a word. */
YRSS_SYN_FN uint32_t yrss_be16_at(uint32_t v, unsigned o)
{
    return (((v >> 8) & 0xffu) << (8u * o)) | ((v & 0xffu) << (8u * (o + 1u)));
}

/* Big-endian u32 as a little-endian word (network byte order in memory). */
YRSS_SYN_FN uint32_t yrss_be32_word(uint32_t v)
{
    return ((v >> 24) & 0xffu) | (((v >> 16) & 0xffu) << 8) |
           (((v >> 8) & 0xffu) << 16) | ((v & 0xffu) << 24);
}

YRSS_SYN_FN uint32_t yrss_synth_flow_of(const struct yrss_synth_params *p, uint64_t i)
{
    uint64_t h = yrss_mix64(p->seed ^ (i * 0xD1B54A32D192ED03ull));
    uint32_t nf = p->nflows ? p->nflows : 1u;
    return (uint32_t)(((h >> 32) * (uint64_t)nf) >> 32);
}

/* IPv4 frame, IHL=5, 14-byte Ethernet header.  proto 6 (TCP) or 17 (UDP). */
YRSS_SYN_FN void yrss_synth_ipv4(uint32_t w[20], uint32_t saddr, uint32_t daddr,
                                 uint32_t sport, uint32_t dport, uint32_t proto,
                                 uint32_t ip_total_len, uint32_t ipid,
                                 uint64_t pay)
{
    w[0] = 0x00000002u;                         /* dst 02:00:00:00:00:02 */
    w[1] = 0x00020200u;                         /* ...   src 02:00:..   */
    w[2] = 0x01000000u;                         /* ...:00:01            */
    w[3] = 0x08u | (0x00u << 8) | (0x45u << 16); /* 0x0800, ver4 IHL5, tos 0 */
    w[4] = yrss_be16_at(ip_total_len & 0xffffu, 0) | yrss_be16_at(ipid & 0xffffu, 2);
    w[5] = 0x40u | (64u << 16) | ((proto & 0xffu) << 24);  /* DF, ttl 64, proto */
    /* bytes 24,25 checksum (left 0: the dispatcher never checks it) */
    w[6] = (((saddr >> 24) & 0xffu) << 16) | (((saddr >> 16) & 0xffu) << 24);
    w[7] = ((saddr >> 8) & 0xffu) | ((saddr & 0xffu) << 8) |
           (((daddr >> 24) & 0xffu) << 16) | (((daddr >> 16) & 0xffu) << 24);
    w[8] = ((daddr >> 8) & 0xffu) | ((daddr & 0xffu) << 8) | yrss_be16_at(sport, 2);
    w[9] = yrss_be16_at(dport, 0);
    if (proto == 17u) {
        w[9] |= yrss_be16_at((ip_total_len - 20u) & 0xffffu, 2);  /* UDP length */
        w[10] = 0;                                                  /* UDP csum 0 */
    } else {
        uint32_t seq = (uint32_t)pay, ack = (uint32_t)(pay >> 32);
        w[9] |= ((seq >> 24) & 0xffu) << 16 | ((seq >> 16) & 0xffu) << 24;
        w[10] = ((seq >> 8) & 0xffu) | ((seq & 0xffu) << 8) |
                ((ack >> 24) & 0xffu) << 16 | ((ack >> 16) & 0xffu) << 24;
        w[11] = ((ack >> 8) & 0xffu) | ((ack & 0xffu) << 8) | (0x50u << 16) | (0x10u << 24);
        w[12] = yrss_be16_at(0xffffu, 0);       /* window 65535, csum 0 */
        w[13] = 0;                              /* urg 0 | payload      */
    }
}

/* Fill the 80-byte window of packet i and its data_len. */
YRSS_SYN_FN void yrss_synth_window(const struct yrss_synth_params *p, uint64_t i,
                                   uint32_t w[20], uint16_t *len_out)
{
    const uint64_t pay = yrss_mix64(p->seed ^ 0xA5A5A5A5ull ^ (i << 1));
    for (int k = 0; k < 20; ++k)
        w[k] = (uint32_t)(pay >> (k & 31)) ^ ((uint32_t)k * 0x9E3779B9u);

    const uint32_t prof = p->profile;
    if (prof == YRSS_SYN_FUZZ) {
        for (int k = 0; k < 20; ++k)
            w[k] = (uint32_t)yrss_mix64(pay + (uint64_t)k * 0x632BE59BD9B4E019ull);
        const uint64_t r = yrss_mix64(pay ^ 0x1234567ull);
        uint32_t et;
        switch ((uint32_t)(r & 15u)) {
        case 10: et = 0x88A8u; break;
        case 11: et = 0x0806u; break;
        case 12: et = 0x8035u; break;
        case 13: et = 0x86DDu; break;
        case 14: et = 0x8100u; break;
        case 15: et = (uint32_t)(r >> 48) & 0xffffu; break;
        default: et = 0x0800u; break;
        }
        uint32_t b14 = (uint32_t)(r >> 8) & 0xffu;
        if (((r >> 16) & 1u) == 0u) b14 = 0x45u;              /* half well-formed */
        uint32_t pr;
        const uint32_t rp = (uint32_t)((r >> 20) % 20u);
        if (rp < 12u) pr = 6u; else if (rp < 16u) pr = 17u;
        else if (rp < 17u) pr = 4u; else pr = (uint32_t)(r >> 40) & 0xffu;
        w[3] = (w[3] & 0xff000000u) | yrss_be16_at(et, 0) | (b14 << 16);
        w[5] = (w[5] & 0x00ffffffu) | (pr << 24);
        const uint32_t rl = (uint32_t)((r >> 28) % 10u);
        const uint32_t lv = (uint32_t)(r >> 32);
        uint32_t L;
        if (rl < 4u) L = 64u;
        else if (rl < 7u) L = lv % 101u;        /* 0..100: every length check */
        else if (rl < 9u) L = lv % 2049u;       /* up to one 2 KB mbuf        */
        else L = lv & 0xffffu;                  /* any u16                    */
        *len_out = (uint16_t)L;
        return;
    }

    if (prof == YRSS_SYN_UDP4_1FLOW) {
        yrss_synth_ipv4(w, 0x0A000001u, 0x0A000002u, 1234u, 5678u, 17u, 50u,
                        (uint32_t)i, pay);
        *len_out = 64;
        return;
    }

    const uint32_t f = yrss_synth_flow_of(p, i);
    const uint64_t h0 = yrss_mix64(p->seed ^ 0x5851F42D4C957F2Dull ^ ((uint64_t)f << 20));
    const uint64_t h1 = yrss_mix64(h0 ^ 0x14057B7EF767814Full);
    const uint32_t saddr = (uint32_t)h0, daddr = (uint32_t)(h0 >> 32);
    const uint32_t sport = (uint32_t)h1 & 0xffffu, dport = (uint32_t)(h1 >> 16) & 0xffffu;
    const uint32_t ipid = (uint32_t)i & 0xffffu;

    if (prof == YRSS_SYN_VLAN6_TCP) {
        const uint64_t h2 = yrss_mix64(h1 ^ 0xDA942042E4DD58B5ull);
        const uint64_t h3 = yrss_mix64(h2 ^ 0x2545F4914F6CDD1Dull);
        w[0] = 0x00000002u; w[1] = 0x00020200u; w[2] = 0x01000000u;
        /* 12-13 0x8100, 14-15 TCI (pcp 0, vid from flow) */
        w[3] = yrss_be16_at(0x8100u, 0) | yrss_be16_at((uint32_t)(h1 >> 32) & 0x0fffu, 2);
        /* 16-17 0x86DD, 18-19 ver6/tc/flow */
        w[4] = yrss_be16_at(0x86DDu, 0) | (0x60u << 16);
        /* 20-21 flow, 22-23 payload length (6: the 64B frame truncates TCP) */
        w[5] = yrss_be16_at(6u, 2);
        /* 24 next header TCP, 25 hop limit, 26..41 src, 42..57 dst */
        w[6] = 6u | (64u << 8) | (0x20u << 16) | (0x01u << 24);        /* 2001:0db8:: */
        w[7] = 0x0du | (0xb8u << 8) | (((uint32_t)h2 & 0xffffu) << 16);
        w[8] = (uint32_t)(h2 >> 16);
        w[9] = (uint32_t)(h2 >> 48) | ((saddr & 0xffffu) << 16);
        w[10] = (saddr >> 16) | (0x20u << 16) | (0x01u << 24);          /* dst 2001:0db8:: */
        w[11] = 0x0du | (0xb8u << 8) | (((uint32_t)h3 & 0xffffu) << 16);
        w[12] = (uint32_t)(h3 >> 16);
        w[13] = (uint32_t)(h3 >> 48) | ((daddr & 0xffffu) << 16);
        w[14] = (daddr >> 16) | yrss_be16_at(sport, 2);                 /* 58-59 sport */
        w[15] = yrss_be16_at(dport, 0) | (w[15] & 0xffff0000u);         /* 60-61 dport */
        *len_out = 64;
        return;
    }

    uint32_t proto = 17u, frame = 64u, dlen = 64u;
    if (prof == YRSS_SYN_TCP4) {
        proto = 6u;
    } else if (prof == YRSS_SYN_JUMBO_TCP4) {
        proto = 6u; frame = 9000u; dlen = 2048u;   /* RTE_MBUF_DEFAULT_DATAROOM */
    } else if (prof == YRSS_SYN_IMIX) {
        const uint32_t r = (uint32_t)((pay >> 40) % 12u);
        frame = r < 7u ? 64u : (r < 11u ? 570u : 1500u);
        dlen = frame;
        proto = ((h1 >> 63) & 1u) ? 6u : 17u;
    }
    yrss_synth_ipv4(w, saddr, daddr, sport, dport, proto, frame - 14u, ipid, pay);
    *len_out = (uint16_t)dlen;
}

#ifdef __cplusplus
}
#endif
#endif /* YRSS_SYNTH_H */
