"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes loader for oracle/liboracle.so (the C restatement in yrss_oracle.c)
and, when present, oracle/_ref/libref_thash.so (the reference's own
toeplitz_hash compiled by build_ref.sh).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
REF_LIB = HERE / "_ref" / "libref_thash.so"
REF_KNI_LIB = HERE / "_ref" / "libref_kni.so"

MLX_KEY = bytes.fromhex(
    "d181c62cf7f4db5b1983a2fc943e1adbd9389e6bd1039c2ca74499ad593d56d9f3253c062adc1ffc")


class OracleCfg(ctypes.Structure):
    _fields_ = [
        ("key", ctypes.c_uint8 * 40),
        ("keylen", ctypes.c_uint32),
        ("nb_procs", ctypes.c_int32),
        ("nb_queues", ctypes.c_uint16),
        ("soft_dispatch", ctypes.c_uint8),
        ("dispatch_only_core", ctypes.c_uint8),
    ]


class SynthParams(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("profile", ctypes.c_uint32),
                ("nflows", ctypes.c_uint32)]


_lib = None
_ref = None
_ref_kni = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE), "all"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = ctypes.CDLL(str(LIB))
        vp, u32 = ctypes.c_void_p, ctypes.c_uint32
        L.oracle_toeplitz_hash.restype = u32
        L.oracle_toeplitz_hash.argtypes = [ctypes.c_uint, ctypes.c_char_p, ctypes.c_uint,
                                           ctypes.c_char_p]
        L.oracle_toeplitz_dispatch.restype = ctypes.c_int
        L.oracle_toeplitz_dispatch.argtypes = [ctypes.c_char_p, ctypes.c_uint16,
                                               ctypes.POINTER(OracleCfg),
                                               ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_dispatch_windows.restype = None
        L.oracle_dispatch_windows.argtypes = [vp, u32, vp, u32, ctypes.POINTER(OracleCfg), vp,
                                              vp, ctypes.c_int]
        L.oracle_process_burst.restype = None
        L.oracle_process_burst.argtypes = [vp, u32, ctypes.c_uint16, vp, vp]
        L.oracle_ff_rss_check.restype = ctypes.c_int
        L.oracle_ff_rss_check.argtypes = [ctypes.POINTER(OracleCfg), ctypes.c_uint16,
                                          ctypes.c_uint16, ctypes.c_uint16, u32, u32,
                                          ctypes.c_uint16, ctypes.c_uint16]
        L.oracle_synth.restype = None
        L.oracle_synth.argtypes = [ctypes.POINTER(SynthParams), ctypes.c_uint64, u32, vp, u32, vp]
        L.oracle_kni_set_bitmap.restype = None
        L.oracle_kni_set_bitmap.argtypes = [ctypes.c_char_p, vp]
        L.oracle_protocol_filter.restype = ctypes.c_int
        L.oracle_protocol_filter.argtypes = [ctypes.c_char_p, ctypes.c_uint16, u32, ctypes.c_int,
                                             vp, vp]
        L.oracle_filter_windows.restype = None
        L.oracle_filter_windows.argtypes = [vp, u32, vp, u32, ctypes.c_int, vp, vp, vp]
        L.oracle_rss_check_batch.restype = None
        L.oracle_rss_check_batch.argtypes = [ctypes.POINTER(OracleCfg), vp, u32, ctypes.c_uint16,
                                             ctypes.c_uint16, ctypes.c_uint16, vp, vp]
        L.oracle_bench_dispatch.restype = ctypes.c_uint64
        L.oracle_bench_dispatch.argtypes = [vp, u32, vp, u32, ctypes.POINTER(OracleCfg), u32,
                                            ctypes.c_int]
        L.oracle_bench_window.restype = ctypes.c_uint64
        L.oracle_bench_window.argtypes = [vp, u32, vp, u32, ctypes.POINTER(OracleCfg),
                                          ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                          ctypes.c_uint64, vp]
        _lib = L
    return _lib


def ref_kni():
    """The reference's compiled kni_set_bitmap / get_bitmap (oracle/_ref,
    fs/lib/ff_dpdk_kni.c:51-123), or None if oracle/_ref is absent."""
    global _ref_kni
    if _ref_kni is None and REF_KNI_LIB.exists():
        R = ctypes.CDLL(str(REF_KNI_LIB))
        R.ref_kni_set_bitmap.restype = None
        R.ref_kni_set_bitmap.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
        R.ref_get_bitmap.restype = ctypes.c_int
        R.ref_get_bitmap.argtypes = [ctypes.c_uint16, ctypes.c_void_p]
        _ref_kni = R
    return _ref_kni


def ref_kni_bitmap(ports: str | None) -> np.ndarray:
    """The 8 KiB bitmap the reference's kni_set_bitmap builds from a port list."""
    bm = np.zeros(8192, np.uint8)
    ref_kni().ref_kni_set_bitmap(None if ports is None else ports.encode(), bm.ctypes.data)
    return bm


def ref_ini_events(path: str):
    """(events, error) of the reference's own INI reader (inih, fs/lib/
    ff_ini_parser.c compiled by build_ref.sh) over a file, recording every
    (section, name, value) it hands the handler; None if oracle/_ref is absent."""
    lib_path = HERE / "_ref" / "libref_ini.so"
    if not lib_path.exists():
        return None
    R = ctypes.CDLL(str(lib_path))
    H = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p,
                         ctypes.c_char_p)
    ev = []

    def rec(_user, s, n, v):
        ev.append((s.decode("latin-1"), n.decode("latin-1"), v.decode("latin-1")))
        return 1

    cb = H(rec)
    R.ini_parse.restype = ctypes.c_int
    R.ini_parse.argtypes = [ctypes.c_char_p, H, ctypes.c_void_p]
    err = R.ini_parse(str(path).encode(), cb, None)
    return ev, err


def ref():
    """The reference's compiled toeplitz_hash, or None if oracle/_ref is absent."""
    global _ref
    if _ref is None and REF_LIB.exists():
        R = ctypes.CDLL(str(REF_LIB))
        R.ref_toeplitz_hash.restype = ctypes.c_uint32
        R.ref_toeplitz_hash.argtypes = [ctypes.c_uint, ctypes.c_char_p, ctypes.c_uint,
                                        ctypes.c_char_p]
        R.ref_default_rsskey.restype = ctypes.POINTER(ctypes.c_uint8)
        _ref = R
    return _ref


def cfg(nb_procs=3, nb_queues=None, soft_dispatch=1, dispatch_only_core=1,
        key: bytes = MLX_KEY) -> OracleCfg:
    c = OracleCfg()
    ctypes.memmove(c.key, key, len(key))
    c.keylen = len(key)
    c.nb_procs = nb_procs
    c.nb_queues = nb_procs if nb_queues is None else nb_queues
    c.soft_dispatch = soft_dispatch
    c.dispatch_only_core = dispatch_only_core
    return c


def toeplitz_hash(data: bytes, key: bytes = MLX_KEY) -> int:
    return lib().oracle_toeplitz_hash(len(key), key, len(data), data)


def toeplitz_dispatch(frame: bytes, length: int, c: OracleCfg) -> tuple[int, int]:
    h = ctypes.c_uint32()
    buf = bytes(frame) + bytes(max(0, 80 - len(frame)))
    q = lib().oracle_toeplitz_dispatch(buf, length, ctypes.byref(c), ctypes.byref(h))
    return q, h.value


def dispatch_windows(win: np.ndarray, stride: int, lens: np.ndarray, c: OracleCfg,
                     fast: bool = True):
    n = int(lens.size)
    win = np.ascontiguousarray(win, dtype=np.uint8)
    lens = np.ascontiguousarray(lens).view(np.uint16)
    q = np.empty(max(n, 1), np.int16)
    h = np.empty(max(n, 1), np.uint32)
    lib().oracle_dispatch_windows(win.ctypes.data, stride, lens.ctypes.data, n, ctypes.byref(c),
                                  q.ctypes.data, h.ctypes.data, 1 if fast else 0)
    return q[:n], h[:n]


def process_burst(q: np.ndarray, nb_queues: int):
    n = int(q.size)
    q = np.ascontiguousarray(q, dtype=np.int16)
    qi = np.empty(max(n, 1), np.uint32)
    qs = np.empty(nb_queues + 2, np.uint32)
    lib().oracle_process_burst(q.ctypes.data, n, nb_queues, qi.ctypes.data, qs.ctypes.data)
    return qi[:n], qs


def synth(profile: int, n: int, first: int = 0, seed: int = 0x9E3779B97F4A7C15,
          nflows: int = 1 << 20, stride: int = 64):
    win = np.empty(max(n, 1) * stride, np.uint8)
    lens = np.empty(max(n, 1), np.uint16)
    p = SynthParams(seed & 0xFFFFFFFFFFFFFFFF, profile, nflows)
    lib().oracle_synth(ctypes.byref(p), first, n, win.ctypes.data, stride, lens.ctypes.data)
    return win[:n * stride], lens[:n]


def bench_dispatch(win, stride, lens, c: OracleCfg, reps: int, fast: bool = False) -> int:
    lens = np.ascontiguousarray(lens).view(np.uint16)
    return lib().oracle_bench_dispatch(win.ctypes.data, stride, lens.ctypes.data, int(lens.size),
                                       ctypes.byref(c), reps, 1 if fast else 0)


def bench_window(win, stride, lens, c: OracleCfg, fast: bool, fnptr: bool, start_ns: int,
                 end_ns: int):
    """Dispatch passes over the sample from CLOCK_MONOTONIC start_ns until
    end_ns (time.monotonic_ns()), inlined or through the registered-dispatcher
    function pointer (ff_dpdk_if.c:1078-1079).  (packets, first ns, last ns)."""
    lens = np.ascontiguousarray(lens).view(np.uint16)
    out = np.zeros(3, np.uint64)
    lib().oracle_bench_window(win.ctypes.data, stride, lens.ctypes.data, int(lens.size),
                              ctypes.byref(c), 1 if fast else 0, 1 if fnptr else 0,
                              start_ns, end_ns, out.ctypes.data)
    return int(out[0]), int(out[1]), int(out[2])


def kni_bitmap(ports: str | None) -> np.ndarray:
    bm = np.zeros(8192, np.uint8)
    lib().oracle_kni_set_bitmap(None if ports is None else ports.encode(), bm.ctypes.data)
    return bm


def protocol_filter(frame: bytes, length: int, enable_kni: bool, tcp_bm, udp_bm,
                    avail: int = 1 << 20) -> int:
    buf = bytes(frame) + bytes(max(0, 80 - len(frame)))
    return lib().oracle_protocol_filter(buf, length, min(avail, len(buf)), 1 if enable_kni else 0,
                                        tcp_bm.ctypes.data, udp_bm.ctypes.data)


def filter_windows(win, stride, lens, enable_kni, tcp_bm, udp_bm) -> np.ndarray:
    n = int(lens.size)
    win = np.ascontiguousarray(win, dtype=np.uint8)
    lens = np.ascontiguousarray(lens).view(np.uint16)
    out = np.empty(max(n, 1), np.int8)
    lib().oracle_filter_windows(win.ctypes.data, stride, lens.ctypes.data, n,
                                1 if enable_kni else 0, tcp_bm.ctypes.data, udp_bm.ctypes.data,
                                out.ctypes.data)
    return out[:n]


def process_packets_route(q, fclass, nb_queues, queue_id, kni_enable, kni_accept, kni_primary,
                          ring_free, clone_ok=lambda i, j: True):
    """Pure-Python restatement of process_packets (ff_dpdk_if.c:1058-1140) for
    a burst from the NIC (pkts_from_ring = 0), one packet at a time, small
    bursts only.  ring_free[j] = free slots of dispatch_ring[port][j].
    Returns (rings: {j: [obj]}, local: [obj], kni: [obj], freed: [obj]) where
    obj = ("pkt", i) or ("clone", i, j)."""
    rings = {j: [] for j in range(nb_queues)}
    local, kni, freed = [], [], []
    free = list(ring_free)
    for i, ret in enumerate(q):
        ret = int(ret)
        if ret < 0 or ret >= nb_queues:
            freed.append(("pkt", i))
            continue
        if ret != queue_id:
            if free[ret] > 0:
                rings[ret].append(("pkt", i))
                free[ret] -= 1
            else:
                freed.append(("pkt", i))
            continue
        f = int(fclass[i])
        if f == 1:                                   # FILTER_ARP
            for j in range(nb_queues):
                if j == queue_id:
                    continue
                if clone_ok(i, j):
                    if free[j] > 0:
                        rings[j].append(("clone", i, j))
                        free[j] -= 1
                    else:
                        freed.append(("clone", i, j))
            if kni_enable and kni_primary and clone_ok(i, 0xFFFF):
                kni.append(("clone", i, 0xFFFF))
            local.append(("pkt", i))
        elif kni_enable and ((f == 2 and kni_accept) or (f == -1 and not kni_accept)):
            kni.append(("pkt", i))
        else:
            local.append(("pkt", i))
    return rings, local, kni, freed


def rss_check_batch(tuples: np.ndarray, nb_queues: int, reta_size: int, queueid: int,
                    key: bytes = MLX_KEY):
    """ff_rss_check over raw 12-byte tuples (uint8 array, n x 12)."""
    t = np.ascontiguousarray(tuples, dtype=np.uint8).reshape(-1, 12)
    n = t.shape[0]
    ok = np.empty(max(n, 1), np.uint8)
    h = np.empty(max(n, 1), np.uint32)
    c = cfg(8, 8, 1, 0, key=key)
    lib().oracle_rss_check_batch(ctypes.byref(c), t.ctypes.data, n, nb_queues, reta_size, queueid,
                                 ok.ctypes.data, h.ctypes.data)
    return ok[:n], h[:n]


def pcap_bytes(frames, ts_sec=None, ts_usec=None, header: bool = True) -> bytes:
    """Restatement of ff_enable_pcap + ff_dump_packets (fs/lib/ff_dpdk_pcap.c:49-102):
    file header {0xA1B2C3D4, 2, 4, 0, 0, 65535, 1}, then per packet
    {sec, usec, caplen = pkt_len, len = pkt_len} + the segment bytes."""
    import struct

    out = bytearray()
    if header:
        out += struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 0xFFFF, 1)
    for i, f in enumerate(frames):
        s = 0 if ts_sec is None else int(ts_sec[i])
        u = 0 if ts_usec is None else int(ts_usec[i])
        out += struct.pack("<IIII", s, u, len(f), len(f)) + bytes(f)
    return bytes(out)
