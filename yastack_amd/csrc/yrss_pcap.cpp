// yrss_pcap.cpp — libpcap 2.4 capture I/O for the soft-RSS engine (SURVEY §8(f)
// rank 3).  Host-only file I/O; no HIP calls.
//
// Writer: the byte layout of F-Stack's per-port pcap dump — ff_enable_pcap
// writes the 24-byte file header (magic 0xA1B2C3D4, v2.4, thiszone 0, sigfigs 0,
// snaplen 65535, linktype 1 = Ethernet) and ff_dump_packets appends one
// 16-byte record header {sec, usec, caplen = pkt_len, len = pkt_len} plus the
// packet bytes per RX mbuf (fs/lib/ff_dpdk_pcap.c:32-102).  Here a whole burst
// is written per call instead of fopen/fclose per packet.
//
// Reader: the replay side — records become header windows + data_len in the
// yrss_dispatch_dev layout, so captures (or the writer's own output) feed the
// GPU path and the oracle identically.
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "yrss.h"

namespace {

struct FileHdr {
    uint32_t magic;
    uint16_t version_major;
    uint16_t version_minor;
    int32_t thiszone;
    uint32_t sigfigs;
    uint32_t snaplen;
    uint32_t linktype;
};
static_assert(sizeof(FileHdr) == 24, "pcap file header is 24 bytes");

struct RecHdr {
    uint32_t sec;
    uint32_t usec;
    uint32_t caplen;
    uint32_t len;
};
static_assert(sizeof(RecHdr) == 16, "pcap record header is 16 bytes");

uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

struct Closer {
    FILE *f;
    ~Closer() { if (f) fclose(f); }
};

}  // namespace

extern "C" {

int yrss_pcap_write(const char *path, int append, const uint8_t *const *data,
                    const uint32_t *len, uint32_t n, const uint32_t *ts_sec,
                    const uint32_t *ts_usec)
{
    if (!path || (n && (!data || !len)))
        return -EINVAL;
    Closer fc{fopen(path, append ? "ab" : "wb")};
    if (!fc.f)
        return -errno;
    if (!append) {
        const FileHdr h = {0xA1B2C3D4u, 2, 4, 0, 0, 0x0000FFFFu, 1u};
        if (fwrite(&h, sizeof(h), 1, fc.f) != 1)
            return -EIO;
    }
    for (uint32_t i = 0; i < n; ++i) {
        const RecHdr r = {ts_sec ? ts_sec[i] : 0u, ts_usec ? ts_usec[i] : 0u, len[i], len[i]};
        if (fwrite(&r, sizeof(r), 1, fc.f) != 1)
            return -EIO;
        if (len[i] && fwrite(data[i], len[i], 1, fc.f) != 1)
            return -EIO;
    }
    return fflush(fc.f) == 0 ? 0 : -EIO;
}

int yrss_pcap_read(const char *path, uint64_t first, uint32_t max, uint8_t *win,
                   uint32_t stride, uint16_t *len, uint32_t *wire_len)
{
    if (!path || (max && (!win || !len)) || stride < YRSS_WIN_MIN)
        return -EINVAL;
    Closer fc{fopen(path, "rb")};
    if (!fc.f)
        return -errno;
    FileHdr h;
    if (fread(&h, sizeof(h), 1, fc.f) != 1)
        return -EIO;
    bool swap;
    switch (h.magic) {
    case 0xA1B2C3D4u: case 0xA1B23C4Du: swap = false; break;   // usec / nsec, native
    case 0xD4C3B2A1u: case 0x4D3CB2A1u: swap = true; break;
    default: return -EINVAL;
    }
    const uint32_t linktype = swap ? bswap32(h.linktype) : h.linktype;
    if ((linktype & 0x0FFFFFFFu) != 1u)                          // LINKTYPE_ETHERNET
        return -EINVAL;
    uint8_t buf[YRSS_WIN_FULL + 2048];
    uint64_t rec = 0;
    uint32_t got = 0;
    while (got < max || max == 0) {
        RecHdr r;
        if (fread(&r, sizeof(r), 1, fc.f) != 1)
            break;                                               // end of capture
        uint32_t cap = swap ? bswap32(r.caplen) : r.caplen;
        const uint32_t wire = swap ? bswap32(r.len) : r.len;
        if (cap > (1u << 26))
            return -EINVAL;                                      // corrupt record
        if (rec++ < first || max == 0) {
            if (fseek(fc.f, cap, SEEK_CUR) != 0)
                return -EIO;
            if (max == 0)
                ++got;                                           // count-only mode
            continue;
        }
        // one record = one single-segment mbuf: data_len = min(caplen, 65535)
        const uint32_t keep = std::min<uint32_t>(cap, stride);
        uint8_t *dst = win + (size_t)got * stride;
        uint32_t done = 0;
        while (done < keep) {
            const uint32_t k = std::min<uint32_t>(keep - done, sizeof(buf));
            if (fread(buf, 1, k, fc.f) != k)
                return -EIO;
            memcpy(dst + done, buf, k);
            done += k;
        }
        if (keep < stride)
            memset(dst + keep, 0, stride - keep);
        if (cap > keep && fseek(fc.f, cap - keep, SEEK_CUR) != 0)
            return -EIO;
        len[got] = (uint16_t)std::min<uint32_t>(cap, 0xFFFFu);
        if (wire_len)
            wire_len[got] = wire;
        ++got;
    }
    return (int)got;
}

}  // extern "C"
