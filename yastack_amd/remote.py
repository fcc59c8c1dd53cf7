"""The soft-RSS engine in a helper process (include/yrss_remote.h).

An F-Stack lcore that hands its bursts to the GPU must survive a GPU fault:
a poisoned HIP context cannot be recovered in the process that owns it, and a
process that touched the GPU cannot be re-executed.  RemoteRss keeps every HIP
call in a ``yrss_helper`` child process: the lcore copies each burst's header
windows into a shared ring, the helper's persistent GPU worker classifies them
in place, and when the helper dies the next poll says so (-EPIPE) and
``restart()`` brings up a fresh helper that finishes the queued bursts.
This module loads only ``libyrss_remote.so`` (no HIP).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

from . import abi

LIB_PATH = abi.PKG_DIR / "_lib" / "libyrss_remote.so"
HELPER_PATH = abi.PKG_DIR / "_lib" / "yrss_helper"

_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_PROTOS = {
    "yrss_remote_start": (ctypes.c_int, [ctypes.POINTER(abi.Config), ctypes.c_char_p, _u32, _u32,
                                         _u32, _u32, ctypes.POINTER(_vp)]),
    "yrss_remote_submit": (ctypes.c_int, [_vp, _vp, _vp, _u32, ctypes.POINTER(ctypes.c_uint64)]),
    "yrss_remote_poll": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_int, _vp, _vp, _vp, _vp]),
    "yrss_remote_restart": (ctypes.c_int, [_vp]),
    "yrss_remote_pid": (ctypes.c_int, [_vp]),
    "yrss_remote_stop": (ctypes.c_int, [_vp]),
}
_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise abi.YrssLibraryError(f"{LIB_PATH} not found: run __graft_entry__.build()")
        lib = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in _PROTOS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


class RemoteRss:
    """One helper process, one ring (yrss_remote_*)."""

    def __init__(self, cfg: abi.Config, nslots: int = 16, max_burst: int = 1024,
                 nblocks: int = 4, timeout_ms: int = 10000, helper: str | None = None):
        self._lib = load()
        self.nb_queues = int(cfg.nb_queues)
        r = _vp()
        path = (helper or str(HELPER_PATH)).encode()
        abi.check(self._lib.yrss_remote_start(ctypes.byref(cfg), path, nslots, max_burst, nblocks,
                                              timeout_ms, ctypes.byref(r)), "yrss_remote_start")
        self._r = r
        self._keep = {}

    @property
    def pid(self) -> int:
        return int(self._lib.yrss_remote_pid(self._r))

    def submit(self, frames) -> int:
        """Copy a burst's windows into the ring; returns its ticket."""
        bufs = [np.frombuffer(bytes(f), dtype=np.uint8) if len(f) else np.zeros(1, np.uint8)
                for f in frames]
        ptrs = np.array([b.ctypes.data for b in bufs], dtype=np.uint64)
        lens = np.array([len(f) for f in frames], dtype=np.uint16)
        t = ctypes.c_uint64()
        rc = self._lib.yrss_remote_submit(self._r, ptrs.ctypes.data, lens.ctypes.data, len(frames),
                                          ctypes.byref(t))
        abi.check(rc, "yrss_remote_submit")
        self._keep[t.value] = len(frames)
        return t.value

    def poll(self, ticket: int, wait: bool = True):
        """(rc, q, hash, qidx, qstart): rc 0 with the outputs, or -errno
        (-EAGAIN pending, -EPIPE helper gone, -ETIMEDOUT no progress)."""
        n = self._keep.get(ticket, 0)
        q = np.empty(max(n, 1), np.int16)
        h = np.empty(max(n, 1), np.uint32)
        qi = np.empty(max(n, 1), np.uint32)
        qs = np.empty(self.nb_queues + 2, np.uint32)
        rc = self._lib.yrss_remote_poll(self._r, ticket, 1 if wait else 0, q.ctypes.data,
                                        h.ctypes.data, qi.ctypes.data, qs.ctypes.data)
        if rc == 0:
            self._keep.pop(ticket, None)
        return rc, q[:n], h[:n], qi[:n], qs

    def restart(self) -> None:
        abi.check(self._lib.yrss_remote_restart(self._r), "yrss_remote_restart")

    def stop(self) -> int:
        rc = 0
        if getattr(self, "_r", None) and self._r.value:
            rc = int(self._lib.yrss_remote_stop(self._r))
            self._r = _vp()
        return rc

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()

    def __del__(self):  # pragma: no cover
        try:
            self.stop()
        except Exception:
            pass


__all__ = ["RemoteRss", "load", "HELPER_PATH", "LIB_PATH", "os"]
