"""Hand-built Ethernet frames for known-answer and edge-case tests.

Layouts follow the reference's DPDK 18.02 headers (rte_ether.h:298-307,
rte_ip.h:31-42, rte_tcp.h:26-36).  Frames are returned padded to at least
80 bytes (YRSS_WIN_FULL) so any window stride up to 80 can be cut from them;
the `length` argument passed alongside is the data_len the dispatcher sees.
"""
from __future__ import annotations

import socket
import struct

ETH_DST = bytes.fromhex("020000000002")
ETH_SRC = bytes.fromhex("020000000001")


def ipv4_frame(src: str, sport: int, dst: str, dport: int, *, proto: int = 6, ihl: int = 5,
               version: int = 4, total_len: int | None = 0, length: int = 64,
               pad_to: int = 80, ports_at_l4: bool = True, ethertype: int = 0x0800) -> bytes:
    """Eth/IPv4 frame; ports at 14+4*IHL when ports_at_l4 and they fit."""
    size = max(length, pad_to)
    b = bytearray(size)
    b[0:6] = ETH_DST
    b[6:12] = ETH_SRC
    struct.pack_into(">H", b, 12, ethertype)
    b[14] = ((version & 0xF) << 4) | (ihl & 0xF)
    tl = (length - 14) if total_len is None else total_len
    struct.pack_into(">H", b, 16, tl & 0xFFFF)
    b[22] = 64
    b[23] = proto
    b[26:30] = socket.inet_aton(src)
    b[30:34] = socket.inet_aton(dst)
    p = 14 + 4 * ihl
    if ports_at_l4 and ihl >= 5 and p + 4 <= size:
        struct.pack_into(">HH", b, p, sport, dport)
    return bytes(b)


def ethertype_frame(ethertype: int, length: int = 64, pad_to: int = 80) -> bytes:
    b = bytearray(max(length, pad_to))
    b[0:6] = ETH_DST
    b[6:12] = ETH_SRC
    struct.pack_into(">H", b, 12, ethertype)
    b[14] = 0x45
    b[23] = 6
    return bytes(b)


def tuple_82599(src: str, dst: str, sport: int, dport: int) -> bytes:
    """Network-order L3+L4 tuple as rte_softrss consumes it (test_thash.c)."""
    return socket.inet_aton(src) + socket.inet_aton(dst) + struct.pack(">HH", sport, dport)
