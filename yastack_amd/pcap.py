"""pcap capture I/O over the C ABI (yrss_pcap_write / yrss_pcap_read).

Mirrors F-Stack's per-port dump format (fs/lib/ff_dpdk_pcap.c:32-102) and
replays captures into the header-window layout of yrss_dispatch_dev, so a
capture feeds the GPU path and the oracle byte-identically.
"""
from __future__ import annotations

import numpy as np

from . import abi


def write(path: str, frames, ts_sec=None, ts_usec=None, append: bool = False) -> None:
    bufs = [np.frombuffer(bytes(f), np.uint8) if len(f) else np.zeros(1, np.uint8)
            for f in frames]
    ptrs = np.array([b.ctypes.data for b in bufs], np.uint64)
    lens = np.array([len(f) for f in frames], np.uint32)
    sec = None if ts_sec is None else np.ascontiguousarray(ts_sec, np.uint32)
    usec = None if ts_usec is None else np.ascontiguousarray(ts_usec, np.uint32)
    rc = abi.load().yrss_pcap_write(path.encode(), 1 if append else 0,
                                    ptrs.ctypes.data if len(frames) else None,
                                    lens.ctypes.data if len(frames) else None, len(frames),
                                    None if sec is None else sec.ctypes.data,
                                    None if usec is None else usec.ctypes.data)
    abi.check(rc, "yrss_pcap_write")


def count(path: str) -> int:
    rc = abi.load().yrss_pcap_read(path.encode(), 0, 0, None, abi.WIN_MIN, None, None)
    abi.check(rc, "yrss_pcap_read")
    return rc


def read(path: str, first: int = 0, max_pkts: int | None = None, stride: int = abi.WIN_FULL):
    """Returns (windows uint8[n*stride], data_len uint16[n], wire_len uint32[n])."""
    n = count(path) - first if max_pkts is None else max_pkts
    n = max(n, 0)
    win = np.zeros(max(n, 1) * stride, np.uint8)
    lens = np.zeros(max(n, 1), np.uint16)
    wire = np.zeros(max(n, 1), np.uint32)
    rc = abi.load().yrss_pcap_read(path.encode(), first, n, win.ctypes.data, stride,
                                   lens.ctypes.data, wire.ctypes.data) if n else 0
    abi.check(rc, "yrss_pcap_read")
    return win[: rc * stride], lens[:rc], wire[:rc]
