"""CPU checks of the oracle's protocol_filter / kni_set_bitmap restatement and
of the pure-Python process_packets routing model.

The reference has no tests for these; every expectation below is derived by
hand from fs/lib/ff_dpdk_kni.c:51-118,218-290 and ff_dpdk_if.c:976-996,
1058-1140 and says which line it exercises.
"""
import struct

import numpy as np

from frames import ethertype_frame, ipv4_frame


def ports_of(bm):
    """Decode an htons-indexed MSB-first bitmap back to host-order ports."""
    out = []
    for idx in np.nonzero(np.unpackbits(bm))[0]:
        idx = int(idx)
        out.append(((idx & 0xFF) << 8) | (idx >> 8))
    return sorted(out)


def test_kni_set_bitmap_rules(oracle_mod):
    assert ports_of(oracle_mod.kni_bitmap("80")) == [80]
    assert ports_of(oracle_mod.kni_bitmap("80,443")) == [80, 443]
    assert ports_of(oracle_mod.kni_bitmap("8000-8003,22")) == [22, 8000, 8001, 8002, 8003]
    # '-' right before ',' is not a range (tail_num < tail - 1 fails): just 80
    assert ports_of(oracle_mod.kni_bitmap("80-,443")) == [80, 443]
    # empty range (lo > hi) sets nothing
    assert ports_of(oracle_mod.kni_bitmap("90-80")) == []
    # values wrap through uint16_t
    assert ports_of(oracle_mod.kni_bitmap("65537")) == [1]
    assert ports_of(oracle_mod.kni_bitmap(None)) == []
    assert len(ports_of(oracle_mod.kni_bitmap("0-70000"))) == 65536


def test_bitmap_bit_order(oracle_mod):
    # set_bitmap(80): p = htons(80) = 0x5000 → byte 0xA00, bit 0x80 (p % 8 == 0)
    bm = oracle_mod.kni_bitmap("80")
    assert bm[0x5000 // 8] == 0x80 and bm.sum() == 0x80
    bm = oracle_mod.kni_bitmap("259")          # htons(259) = 0x0301 → bit 0x40 of byte 0x60
    assert bm[0x0301 // 8] == 0x40


def test_protocol_filter_cases(oracle_mod):
    tcp = oracle_mod.kni_bitmap("80,443")
    udp = oracle_mod.kni_bitmap("53")
    pf = lambda f, L, on=True: oracle_mod.protocol_filter(f, L, on, tcp, udp)  # noqa: E731
    base = ("10.0.0.1", 1234, "10.0.0.2")
    assert pf(ethertype_frame(0x0806), 64) == 1                 # ARP even with KNI off
    assert pf(ethertype_frame(0x0806), 64, on=False) == 1
    assert pf(ethertype_frame(0x0806), 13) == -1                # len < ETHER_HDR_LEN
    assert pf(ethertype_frame(0x8035), 64) == -1                # RARP is not ARP here
    assert pf(ipv4_frame(*base, 80), 64) == 2                   # TCP dport in bitmap
    assert pf(ipv4_frame(*base, 80), 64, on=False) == -1        # !enable_kni
    assert pf(ipv4_frame(*base, 81), 64) == -1
    assert pf(ipv4_frame(*base, 53, proto=17), 64) == 2         # UDP bitmap
    assert pf(ipv4_frame(*base, 80, proto=17), 64) == -1
    assert pf(ipv4_frame(*base, 80), 14 + 20 + 19) == -1        # TCP hdr < 20 bytes
    assert pf(ipv4_frame(*base, 53, proto=17), 14 + 20 + 8) == 2   # UDP hdr = 8 is enough
    assert pf(ipv4_frame(*base, 53, proto=17), 14 + 20 + 7) == -1
    assert pf(ethertype_frame(0x86DD), 64) == -1


def ipip_frame(inner_ihl, inner_proto, dport, outer_ihl=5, length=80):
    b = bytearray(ipv4_frame("10.0.0.1", 1, "10.0.0.2", 2, proto=4, ihl=outer_ihl,
                             length=length, ports_at_l4=False))
    o = 14 + 4 * outer_ihl
    b[o] = 0x40 | inner_ihl
    b[o + 9] = inner_proto
    p = o + 4 * inner_ihl
    if inner_ihl >= 3 and p + 4 <= len(b):      # ports must not overwrite the header
        struct.pack_into(">HH", b, p, 1111, dport)
    return bytes(b)


def test_protocol_filter_ipip(oracle_mod):
    tcp = oracle_mod.kni_bitmap("80")
    udp = oracle_mod.kni_bitmap("53")
    pf = lambda f, L, avail=1 << 20: oracle_mod.protocol_filter(f, L, True, tcp, udp, avail)  # noqa
    assert pf(ipip_frame(5, 6, 80), 80) == 2        # IPIP → inner TCP (ff_dpdk_kni.c:274)
    assert pf(ipip_frame(5, 17, 53), 80) == 2
    assert pf(ipip_frame(5, 6, 81), 80) == -1
    # IHL=0 inner header recurses on itself forever in the reference → LOOP
    assert pf(ipip_frame(0, 4, 0), 80) == -3
    # outer IHL 10: inner TCP dport at bytes 76..77, beyond a 64-byte window →
    # TRUNC (boundary rule); inside an 80-byte window it resolves
    deep = ipip_frame(5, 6, 80, outer_ihl=10, length=100)
    assert pf(deep, 100, avail=64) == -2
    assert pf(deep, 100, avail=80) == 2
    assert pf(deep, 100) == 2


def test_route_model_semantics(oracle_mod):
    # queue_id 0 dispatcher, 3 queues; q: 2,1,0(ARP),5(bad),0,1 ; ring 1 has 1 slot
    q = [2, 1, 0, 5, 0, 1]
    f = [-1, -1, 1, -1, 2, -1]
    rings, local, kni, freed = oracle_mod.process_packets_route(
        q, f, 3, 0, kni_enable=True, kni_accept=True, kni_primary=True, ring_free=[9, 1, 9])
    assert rings[1] == [("pkt", 1)]                 # ring full afterwards
    assert rings[2] == [("pkt", 0), ("clone", 2, 2)]
    assert ("clone", 2, 1) in freed and ("pkt", 5) in freed and ("pkt", 3) in freed
    assert local == [("pkt", 2)]                    # ARP stays local too
    assert kni == [("clone", 2, 0xFFFF), ("pkt", 4)]  # KNI clone of ARP, KNI-accepted pkt


# ---- pinned to the reference itself: oracle/_ref/libref_kni.so is
# fs/lib/ff_dpdk_kni.c:51-123 compiled verbatim by oracle/build_ref.sh ----------

def _ref_or_skip(oracle_mod):
    import pytest

    if oracle_mod.ref_kni() is None:
        pytest.skip("oracle/_ref/libref_kni.so not built (reference not mounted)")


def _random_port_list(rng):
    def num():
        r = rng.random()
        if r < 0.05:
            return str(int(rng.integers(-5, 1)))
        if r < 0.1:
            return str(int(rng.integers(65530, 70001)))
        return str(int(rng.integers(0, 65536)))

    pieces = []
    for _ in range(int(rng.integers(1, 6))):
        k = rng.random()
        if k < 0.4:
            pieces.append(num())
        elif k < 0.7:
            lo = int(rng.integers(0, 65536))
            pieces.append(f"{lo}-{min(lo + int(rng.integers(-3, 300)), 70000)}")
        elif k < 0.76:
            pieces.append(num() + "-")           # '-' right before ',' (tail_num < tail - 1)
        elif k < 0.82:
            pieces.append("-" + num())
        elif k < 0.86:
            pieces.append("")                   # empty field
        elif k < 0.9:
            pieces.append(" " + num())          # atoi skips leading blanks
        elif k < 0.94:
            pieces.append(f"{num()}-{num()}-{num()}")
        else:
            pieces.append(rng.choice(["abc", "0x50", "80a", "-", "--", "8-0-"]))
    return ",".join(pieces)


def test_kni_set_bitmap_vs_reference(oracle_mod):
    _ref_or_skip(oracle_mod)
    fixed = ["80", "80,443", "8000-8080", "80-", "-5", "90-80", "0-70000", "", ",", "80,,443",
             "65535", "65536", "65537", "-1", "1-", "a-b", "1,2-", "5-,7", "0", "10-20,15-25"]
    for s in fixed + [None]:
        assert np.array_equal(oracle_mod.kni_bitmap(s), oracle_mod.ref_kni_bitmap(s)), s
    rng = np.random.default_rng(20261016)
    for _ in range(3000):
        s = _random_port_list(rng)
        assert np.array_equal(oracle_mod.kni_bitmap(s), oracle_mod.ref_kni_bitmap(s)), s


def test_port_lookup_vs_reference_get_bitmap(oracle_mod):
    """protocol_filter's port test (ff_dpdk_kni.c:232-236, 244-248) against the
    reference's get_bitmap on the dst_port as stored (network order read as a
    little-endian uint16)."""
    _ref_or_skip(oracle_mod)
    R = oracle_mod.ref_kni()
    rng = np.random.default_rng(7)
    for trial in range(6):
        spec = _random_port_list(rng)
        tcp = oracle_mod.kni_bitmap(spec)
        udp = oracle_mod.kni_bitmap(_random_port_list(rng))
        ports = list(rng.integers(0, 65536, 300)) + [80, 443, 0, 65535]
        for dport in ports:
            dport = int(dport)
            raw = ((dport & 0xFF) << 8) | (dport >> 8)     # LE read of the network bytes
            for proto, bm in ((6, tcp), (17, udp)):
                f = ipv4_frame("10.0.0.1", 1234, "10.0.0.2", dport, proto=proto)
                want = 2 if R.ref_get_bitmap(raw, bm.ctypes.data) else -1
                assert oracle_mod.protocol_filter(f, 64, True, tcp, udp) == want, (spec, dport)
