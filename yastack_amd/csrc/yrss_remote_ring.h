// yrss_remote_ring.h — the ring shared by an lcore's yrss_remote client
// (yrss_remote.cpp, no HIP) and its yrss_helper process (yrss_helper.cpp, the
// GPU context).  One memfd mapping:
//
//   Header (one page) | Slot[nslots] (client lines) | Done[nslots] (helper
//   lines) | slot data areas
//
// Slot data area (per slot, 256-byte aligned): windows [max_burst][80] |
// len u16[max_burst] | q i16[max_burst] | hash u32[max_burst] |
// qidx u32[max_burst] | qstart u32[nb + 1].  The helper registers the whole
// mapping with the GPU, so the persistent worker reads the windows and writes
// the outputs in place.
//
// Protocol: the client fills a slot's windows and lengths, then publishes
// the ticket in Slot::seq (release).  The helper takes tickets in order from
// Header::first, completes them in order and publishes Done::ticket
// (release) after the outputs; the client reads Done::ticket with acquire.
// A restarted helper resumes at Header::first = the oldest ticket not done.
#ifndef YRSS_REMOTE_RING_H
#define YRSS_REMOTE_RING_H

#include <stddef.h>
#include <stdint.h>

#include "yrss.h"

namespace yrss_ring {

constexpr uint32_t kMagic = 0x59525247u;   // "YRRG"
constexpr uint32_t kVersion = 1;
constexpr uint32_t kWin = YRSS_WIN_FULL;   // window bytes per packet in a slot
constexpr size_t kHeaderBytes = 4096;

struct alignas(64) Header {
    uint32_t magic, version;
    uint32_t nslots, max_burst, nblocks, nb;
    uint64_t slot_bytes;      // bytes of one slot's data area
    uint64_t data_off;        // offset of slot 0's data area
    uint64_t map_bytes;
    uint64_t first;           // the helper's first ticket (restart resumes here)
    uint32_t inject;          // fault injection for tests: 1 = never complete a burst
    uint32_t pad0;
    struct yrss_config cfg;
    alignas(64) uint32_t stop;        // client: leave
    alignas(64) int32_t ready;        // helper: 0 starting, 1 serving, < 0 -errno
    uint32_t pad1;
    uint64_t completed;               // helper: bursts completed (progress)
};
static_assert(sizeof(Header) <= kHeaderBytes, "header fits its page");

struct alignas(64) Slot {
    uint64_t seq;             // client: published ticket (release)
    uint32_t n;
    uint32_t pad[13];
};

struct alignas(64) Done {
    uint64_t ticket;          // helper: completed ticket (release)
    int32_t status;           // 0 or -errno of that burst
    uint32_t pad[13];
};

struct Area {                 // a slot's data area, as offsets from its start
    size_t win, len, q, hash, qidx, qstart, bytes;
};

inline Area area(uint32_t max_burst, uint32_t nb)
{
    auto up = [](size_t x) { return (x + 255u) & ~(size_t)255u; };
    Area a;
    a.win = 0;
    a.len = up(a.win + (size_t)max_burst * kWin);
    a.q = up(a.len + (size_t)max_burst * 2u);
    a.hash = up(a.q + (size_t)max_burst * 2u);
    a.qidx = up(a.hash + (size_t)max_burst * 4u);
    a.qstart = up(a.qidx + (size_t)max_burst * 4u);
    a.bytes = up(a.qstart + ((size_t)nb + 1u) * 4u);
    return a;
}

inline size_t slots_off() { return kHeaderBytes; }
inline size_t done_off(uint32_t nslots) { return kHeaderBytes + (size_t)nslots * sizeof(Slot); }
inline size_t data_off(uint32_t nslots)
{
    return (done_off(nslots) + (size_t)nslots * sizeof(Done) + 4095u) & ~(size_t)4095u;
}

}  // namespace yrss_ring

#endif  // YRSS_REMOTE_RING_H
