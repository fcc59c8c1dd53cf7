"""ctypes binding of the C ABI in include/yrss.h.

The shared library ``yastack_amd/_lib/libyrss.so`` is built in-tree by
``__graft_entry__.build()`` (hipcc --offload-arch=gfx950).  There is no
fallback: if the library is missing, every entry point raises
:class:`YrssLibraryError` — the product path never degrades to a CPU
implementation.
"""
from __future__ import annotations

import ctypes
import errno
import os
import re
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
LIB_PATH = PKG_DIR / "_lib" / "libyrss.so"
# the same sources built with -DYRSS_TEST_HOOKS (include/yrss_test_hooks.h):
# loaded by the GPU tests that drive the fault guards, never by the product
TEST_LIB_PATH = PKG_DIR / "_lib" / "libyrss_test.so"
HEADER_PATH = REPO_DIR / "include" / "yrss.h"

RSS_KEY_LEN = 40
DEFAULT_Q = 2
Q_TRUNCATED = -2
WIN_MIN = 64
WIN_FULL = 80
MAX_QUEUES = 256
MAX_PROCS = 4096
F_WRITE_RSS = 0x1
F_ASYNC = 0x2

K_PARSE_HASH, K_SCAN, K_SCATTER = 0, 1, 2
K_BURST, K_WORKER = 8, 9            # kernel ids of fault records only

# device-side fault record codes (yrss_fault_info)
FAULT_NONE, FAULT_SCAN_TIMEOUT, FAULT_LIST_RANGE, FAULT_COUNT_MISMATCH, FAULT_COUNT_SLOT, \
    FAULT_STAGE, FAULT_LINE_CAPACITY = range(7)

# protocol_filter classes (ff_dpdk_kni.h:34-38) + boundary outcomes
FILTER_UNKNOWN, FILTER_ARP, FILTER_KNI, FILTER_TRUNC, FILTER_LOOP = -1, 1, 2, -2, -3
ROUTE_KNI_QUEUE = 0xFFFF   # queue argument of the clone callback for the KNI clone

# struct rte_mbuf offsets of DPDK 18.02 (dpdk/lib/librte_mbuf/rte_mbuf.h:412-560)
MBUF_OFF_BUF_ADDR = 0
MBUF_OFF_DATA_OFF = 16
MBUF_OFF_DATA_LEN = 40
MBUF_OFF_HASH_RSS = 44

# synthetic profiles (include/yrss_synth.h)
SYN_UDP4_1FLOW, SYN_UDP4, SYN_IMIX, SYN_VLAN6_TCP, SYN_JUMBO_TCP4, SYN_TCP4, SYN_FUZZ = range(7)
SYN_NAMES = {
    SYN_UDP4_1FLOW: "udp4_1flow", SYN_UDP4: "udp4", SYN_IMIX: "imix",
    SYN_VLAN6_TCP: "vlan6_tcp", SYN_JUMBO_TCP4: "jumbo_tcp4", SYN_TCP4: "tcp4",
    SYN_FUZZ: "fuzz",
}


# Fault records (code, kernel, where, value) found unread when a SoftRss
# context closed: tests fail on any entry (tests/conftest.py).
FAULT_LOG: list = []


class YrssLibraryError(RuntimeError):
    """The HIP library is missing or failed to load (no silent fallback)."""


class YrssError(OSError):
    """A C-ABI call returned a negative errno."""


class MbufLayout(ctypes.Structure):
    _fields_ = [
        ("off_buf_addr", ctypes.c_uint16),
        ("off_data_off", ctypes.c_uint16),
        ("off_data_len", ctypes.c_uint16),
        ("off_hash_rss", ctypes.c_uint16),
    ]


class Config(ctypes.Structure):
    _fields_ = [
        ("rss_key", ctypes.c_uint8 * RSS_KEY_LEN),
        ("rss_key_len", ctypes.c_uint32),
        ("nb_procs", ctypes.c_int32),
        ("nb_queues", ctypes.c_uint16),
        ("soft_dispatch", ctypes.c_uint8),
        ("dispatch_only_core", ctypes.c_uint8),
        ("device", ctypes.c_int32),
        ("max_burst", ctypes.c_uint32),
        ("mbuf", MbufLayout),
    ]


class DevBatch(ctypes.Structure):
    _fields_ = [
        ("win", ctypes.c_void_p),
        ("win_stride", ctypes.c_uint32),
        ("n", ctypes.c_uint32),
        ("len", ctypes.c_void_p),
        ("q", ctypes.c_void_p),
        ("hash", ctypes.c_void_p),
        ("qidx", ctypes.c_void_p),
        ("qstart", ctypes.c_void_p),
        ("filter", ctypes.c_void_p),
    ]


ENQUEUE_FN = ctypes.CFUNCTYPE(ctypes.c_uint, ctypes.c_void_p, ctypes.c_uint16,
                              ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint)
CLONE_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint16)
RELEASE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)


class RouteOps(ctypes.Structure):
    _fields_ = [
        ("enqueue", ENQUEUE_FN),
        ("clone", CLONE_FN),
        ("release", RELEASE_FN),
        ("user", ctypes.c_void_p),
    ]


class RouteResult(ctypes.Structure):
    _fields_ = [
        ("n_local", ctypes.c_uint32),
        ("n_kni", ctypes.c_uint32),
        ("n_freed", ctypes.c_uint32),
        ("n_arp", ctypes.c_uint32),
        ("n_unresolved", ctypes.c_uint32),
        ("n_ring", ctypes.c_uint32 * MAX_QUEUES),
    ]


class Fault(ctypes.Structure):
    _fields_ = [
        ("code", ctypes.c_uint32),
        ("kernel", ctypes.c_uint32),
        ("where", ctypes.c_uint32),
        ("value", ctypes.c_uint32),
    ]


class Tuning(ctypes.Structure):
    """Layout overrides (yrss_set_tuning); zero fields are the defaults."""
    _fields_ = [
        ("chunk_tiles", ctypes.c_uint32),
        ("span_tiles", ctypes.c_uint32),
        ("parse_blocks", ctypes.c_uint32),
        ("one_launch", ctypes.c_uint32),
        ("scatter_xcd", ctypes.c_int32),
        ("scan_kernel", ctypes.c_uint32),
    ]


class SynthParams(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("profile", ctypes.c_uint32),
        ("nflows", ctypes.c_uint32),
    ]


_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_PROTOS = {
    "yrss_version": (ctypes.c_char_p, []),
    "yrss_kernel_name": (ctypes.c_char_p, [ctypes.c_int]),
    "yrss_config_default": (None, [ctypes.POINTER(Config)]),
    "yrss_config_validate": (ctypes.c_int, [ctypes.POINTER(Config)]),
    "yrss_init": (ctypes.c_int, [ctypes.POINTER(Config), ctypes.POINTER(_vp)]),
    "yrss_fini": (None, [_vp]),
    "yrss_dispatch_dev": (ctypes.c_int, [_vp, _vp, _u32, _vp, _u32, _vp, _vp, _vp, _vp, _vp]),
    "yrss_dispatch_burst": (ctypes.c_int, [_vp, _vp, _u32, _vp, _vp, _vp, _vp, _u32]),
    "yrss_dispatch_frames": (ctypes.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp]),
    "yrss_synth_dev": (ctypes.c_int, [_vp, ctypes.POINTER(SynthParams), ctypes.c_uint64, _u32,
                                      _vp, _u32, _vp, _vp]),
    "yrss_timing_enable": (ctypes.c_int, [_vp, ctypes.c_int]),
    "yrss_timing_read": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(_u32)]),
    "yrss_timing_quantile": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_double,
                                            ctypes.POINTER(ctypes.c_double)]),
    "yrss_grid_for": (_u32, [_vp, _u32]),
    "yrss_status": (ctypes.c_int, [_vp]),
    "yrss_fault_info": (ctypes.c_int, [_vp, ctypes.POINTER(Fault)]),
    "yrss_set_tuning": (ctypes.c_int, [_vp, ctypes.POINTER(Tuning)]),
    "yrss_wait": (ctypes.c_int, [_vp]),
    "yrss_worker_start": (ctypes.c_int, [_vp, _u32, _u32]),
    "yrss_worker_submit": (ctypes.c_int, [_vp, _vp, _u32, _vp, _vp, _vp, _vp, _u32,
                                          ctypes.POINTER(ctypes.c_uint64)]),
    "yrss_worker_submit_frames": (ctypes.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp,
                                                 ctypes.POINTER(ctypes.c_uint64)]),
    "yrss_worker_submit_windows": (ctypes.c_int, [_vp, _vp, _u32, _vp, _u32, _vp, _vp, _vp, _vp,
                                                  ctypes.POINTER(ctypes.c_uint64)]),
    "yrss_worker_poll": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_int]),
    "yrss_worker_stop": (ctypes.c_int, [_vp]),
    "yrss_dispatch_frames_zc_ex": (ctypes.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp,
                                                  _u32]),
    "yrss_shard_range": (ctypes.c_int, [ctypes.c_uint64, _u32, _u32,
                                        ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.POINTER(ctypes.c_uint64)]),
    "yrss_merge_queue_lists": (ctypes.c_int, [_u32, _u32, _vp, _vp, _vp, _vp, _vp]),
    "yrss_fanout_init": (ctypes.c_int, [ctypes.POINTER(Config), _vp, _u32, _u32, _u32,
                                        ctypes.POINTER(_vp)]),
    "yrss_fanout_fini": (ctypes.c_int, [_vp]),
    "yrss_fanout_size": (_u32, [_vp]),
    "yrss_fanout_register_host_memory": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t]),
    "yrss_fanout_unregister_host_memory": (ctypes.c_int, [_vp, _vp]),
    "yrss_fanout_submit": (ctypes.c_int, [_vp, _vp, _u32, _vp, _vp, _vp, _vp, _u32,
                                          ctypes.POINTER(ctypes.c_uint64)]),
    "yrss_fanout_submit_frames": (ctypes.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp,
                                                 ctypes.POINTER(ctypes.c_uint64)]),
    "yrss_fanout_next": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]),
    "yrss_fanout_route": (ctypes.c_int, [ctypes.c_uint64, _u32, ctypes.POINTER(_u32),
                                         ctypes.POINTER(ctypes.c_uint64)]),
    "yrss_set_dispatch_ctx": (ctypes.c_int, [_vp]),
    "yrss_toeplitz_dispatch": (ctypes.c_int, [_vp, ctypes.c_uint16, ctypes.c_uint16,
                                              ctypes.c_uint16]),
    "yrss_set_kni": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p,
                                    ctypes.c_char_p]),
    "yrss_dispatch_dev_ex": (ctypes.c_int, [_vp, ctypes.POINTER(DevBatch), _vp]),
    "yrss_dispatch_burst_zc": (ctypes.c_int, [_vp, _vp, _u32, _vp, _vp, _vp, _vp, _u32]),
    "yrss_dispatch_frames_zc": (ctypes.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp]),
    "yrss_register_host_memory": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t]),
    "yrss_unregister_host_memory": (ctypes.c_int, [_vp, _vp]),
    "yrss_pcap_write": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, _vp, _vp, _u32, _vp, _vp]),
    "yrss_pcap_read": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint64, _u32, _vp, _u32, _vp,
                                      _vp]),
    "yrss_rss_check_dev": (ctypes.c_int, [_vp, _vp, _u32, ctypes.c_uint16, ctypes.c_uint16,
                                          ctypes.c_uint16, _vp, _vp, _vp]),
    "yrss_rss_lport_sweep": (ctypes.c_int, [_vp, _u32, _u32, ctypes.c_uint16, ctypes.c_uint16,
                                            ctypes.c_uint16, ctypes.c_uint16, _vp]),
    "yrss_route_burst": (ctypes.c_int, [_vp, _vp, _u32, ctypes.c_uint16, ctypes.c_int,
                                        ctypes.POINTER(RouteOps), _vp, _vp,
                                        ctypes.POINTER(RouteResult)]),
}

# include/yrss_test_hooks.h (libyrss_test.so)
_TEST_PROTOS = {
    "yrss_debug_worker_inject": (ctypes.c_int, [_vp, ctypes.c_uint64]),
    "yrss_debug_line_groups": (ctypes.c_int, [_vp, _u32, ctypes.c_int]),
    "yrss_debug_partial_merge": (ctypes.c_int, [_vp, ctypes.c_int]),
}

_lib = None
_libs: dict[str, ctypes.CDLL] = {}


def header_functions(path: Path = HEADER_PATH) -> list[str]:
    """Names of every function declared in include/yrss.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"#define[^\n]*", "", text)
    names = re.findall(r"\b(yrss_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def load(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    """Load libyrss.so (once per path; default YRSS_LIB or the in-tree build).
    Raises YrssLibraryError if it is absent.  Distinct paths load side by side
    (RTLD_LOCAL), which tools/ab_inproc.py uses to compare builds in one
    process."""
    global _lib
    if path is None and _lib is not None:
        return _lib
    p = Path(path if path is not None else os.environ.get("YRSS_LIB", LIB_PATH))
    key = str(p.resolve()) if p.exists() else str(p)
    if key in _libs:
        return _libs[key]
    if not p.exists():
        raise YrssLibraryError(
            f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    try:
        lib = ctypes.CDLL(str(p))
    except OSError as e:  # pragma: no cover - environment specific
        raise YrssLibraryError(f"cannot load {p}: {e}") from e
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    for name, (res, args) in _TEST_PROTOS.items():   # libyrss_test.so only
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
    _libs[key] = lib
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc < 0:
        raise YrssError(-rc, f"{what}: {os.strerror(-rc)} (errno {-rc})")


def default_config() -> Config:
    cfg = Config()
    load().yrss_config_default(ctypes.byref(cfg))
    return cfg


__all__ = [n for n in dir() if not n.startswith("_")] + ["errno"]
