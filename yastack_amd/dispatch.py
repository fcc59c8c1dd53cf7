"""Host-side mirror of yastack's dispatch interface over the HIP engine.

Reference interface (fs/lib/ff_api.h:146-176, fs/lib/ff_dpdk_if.c):

* ``toeplitz_dispatch(data, len, queue_id, nb_queues) -> int`` — per packet.
  Here: :meth:`SoftRss.dispatch_frames` / :meth:`SoftRss.dispatch_burst`
  return the same per-packet ints for a whole burst, computed on the GPU.
* ``process_packets``' dispatcher block (ff_dpdk_if.c:1078-1094) — drop
  ``ret < 0 || ret >= nb_queues``, else enqueue to ``dispatch_ring[port][ret]``.
  Here: the per-queue FIFO index lists of :class:`DispatchResult`.
* ``ff_global_cfg`` knobs (nb_procs, soft_dispatch, dispatch_only_core) and the
  port's nb_queues: the :class:`SoftRss` constructor, or
  :meth:`SoftRss.from_ff_config` for an fs/lib INI file.

Device memory and streams come from PyTorch (plumbing only); every byte of
parse/hash/compaction runs in the HIP kernels of libyrss.so.
"""
from __future__ import annotations

import ctypes
import errno
from dataclasses import dataclass

import numpy as np

from . import abi


@dataclass
class DispatchResult:
    """Per-packet queue/hash plus per-queue FIFO index lists.

    ``q[i]``      toeplitz_dispatch's return for packet i (int16)
    ``hash[i]``   Toeplitz hash (0 where the reference does not hash)
    ``qidx``      packet indices grouped by bucket, FIFO inside a bucket
    ``qstart``    nb_queues+2 offsets; bucket nb_queues = packets the
                  reference frees (ret < 0 or ret >= nb_queues)
    """

    q: object
    hash: object
    qidx: object = None
    qstart: object = None
    filter: object = None     # protocol_filter class per packet (abi.FILTER_*)

    def queue(self, b: int):
        """Indices dispatched to queue b (b == nb_queues: dropped)."""
        s = self.qstart
        return self.qidx[int(s[b]):int(s[b + 1])]


def _check_dev_sizes(n, stride, win, lens, out, nb_queues):
    """The C ABI takes raw device pointers and cannot see the buffers' sizes: a
    batch larger than its buffers would fault the GPU.  Refuse it here."""
    def nbytes(t):
        return 0 if t is None else int(t.numel()) * int(t.element_size())
    if n < 0:
        raise ValueError("negative batch size")
    if n == 0:
        return
    # the kernel may read any byte below the stride of a window (rare header walks)
    need = [("win", win, n * stride), ("lens", lens, 2 * n),
            ("q", out.q, 2 * n)]
    if out.hash is not None:
        need.append(("hash", out.hash, 4 * n))
    if out.qidx is not None:
        need.append(("qidx", out.qidx, 4 * n))
    if out.qstart is not None:
        need.append(("qstart", out.qstart, 4 * (nb_queues + 2)))
    if out.filter is not None:
        need.append(("filter", out.filter, n))
    for name, t, b in need:
        if nbytes(t) < b:
            raise ValueError(f"{name} holds {nbytes(t)} bytes, the batch of {n} needs {b}")


def _ptr(t) -> int | None:
    if t is None:
        return None
    if isinstance(t, np.ndarray):
        return t.ctypes.data
    return t.data_ptr()


class SoftRss:
    """One engine context on one GPU (``yrss_ctx``)."""

    def __init__(self, nb_procs: int = 3, nb_queues: int | None = None,
                 soft_dispatch: int = 1, dispatch_only_core: int = 1,
                 rss_key: bytes | None = None, device: int = 0,
                 max_burst: int = 1 << 16, lib_path: str | None = None):
        self._lib = abi.load(lib_path)
        cfg = abi.Config()
        self._lib.yrss_config_default(ctypes.byref(cfg))
        if rss_key is not None:
            if not 4 <= len(rss_key) <= abi.RSS_KEY_LEN:
                raise ValueError("rss_key must be 4..40 bytes")
            ctypes.memmove(cfg.rss_key, bytes(rss_key), len(rss_key))
            cfg.rss_key_len = len(rss_key)
        cfg.nb_procs = nb_procs
        cfg.nb_queues = nb_procs if nb_queues is None else nb_queues
        cfg.soft_dispatch = soft_dispatch
        cfg.dispatch_only_core = dispatch_only_core
        cfg.device = device
        cfg.max_burst = max_burst
        self.cfg = cfg
        self.nb_queues = int(cfg.nb_queues)
        self.device = device
        ctx = ctypes.c_void_p()
        abi.check(self._lib.yrss_init(ctypes.byref(cfg), ctypes.byref(ctx)), "yrss_init")
        self._ctx = ctx

    @classmethod
    def from_ff_config(cls, path: str, port: int = 0, device: int = 0, **kw) -> "SoftRss":
        from .ffconfig import load_ff_config

        fc = load_ff_config(path)
        eng = cls(nb_procs=fc.nb_procs, nb_queues=fc.nb_queues[port],
                  soft_dispatch=fc.soft_dispatch,
                  dispatch_only_core=fc.dispatch_only_core, device=device, **kw)
        if fc.kni_enable:
            # init_kni (ff_dpdk_if.c:598-606) behind enable_kni (:921-923)
            eng.set_kni(True, fc.kni_method, fc.kni_tcp_port, fc.kni_udp_port)
        return eng

    # -- lifetime ---------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_ctx", None) and self._ctx.value:
            # a device guard that fired and was never read (yrss_status /
            # fault_info) is logged before the context goes (abi.FAULT_LOG);
            # a context that already timed out on the GPU is not waited for
            # again (yrss_fault_info drains the context's streams)
            f = abi.Fault()
            if not getattr(self, "_hung", False) and \
                    self._lib.yrss_fault_info(self._ctx, ctypes.byref(f)) == 0 and f.code:
                abi.FAULT_LOG.append((int(f.code), int(f.kernel), int(f.where), int(f.value)))
            self._lib.yrss_fini(self._ctx)
            self._ctx = ctypes.c_void_p()

    def _ck(self, rc: int, what: str) -> None:
        if rc == -errno.ETIMEDOUT:
            self._hung = True     # close() does not wait on this context again
        abi.check(rc, what)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # -- torch plumbing ------------------------------------------------------
    def _torch(self):
        import torch

        return torch

    def _stream(self, stream):
        torch = self._torch()
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        return ctypes.c_void_p(stream.cuda_stream)

    # -- KNI / protocol_filter ------------------------------------------------
    def set_kni(self, enable: bool, method: str | None = "reject", tcp_ports: str | None = None,
                udp_ports: str | None = None) -> None:
        """ff_kni_init/init_kni: enable, method accept|reject, port lists."""
        enc = (lambda x: None if x is None else x.encode())
        abi.check(self._lib.yrss_set_kni(self._ctx, 1 if enable else 0, enc(method),
                                         enc(tcp_ports), enc(udp_ports)), "yrss_set_kni")

    # -- device-resident path ---------------------------------------------
    def dispatch_dev(self, win, lens, stride: int, n: int | None = None, *,
                     out=None, want_hash: bool = True, compact: bool = True,
                     want_filter: bool = False, stream=None) -> DispatchResult:
        """Classify n packets resident in HBM (``yrss_dispatch_dev_ex``)."""
        n = int(lens.numel()) if n is None else n
        dev = lens.device
        if out is None:
            out = self.alloc_out(n, dev, want_hash, compact, want_filter)
        _check_dev_sizes(n, stride, win, lens, out, self.nb_queues)
        b = abi.DevBatch(_ptr(win), stride, n, _ptr(lens), _ptr(out.q), _ptr(out.hash),
                         _ptr(out.qidx), _ptr(out.qstart), _ptr(out.filter))
        rc = self._lib.yrss_dispatch_dev_ex(self._ctx, ctypes.byref(b), self._stream(stream))
        abi.check(rc, "yrss_dispatch_dev_ex")
        return out

    def alloc_out(self, n: int, dev, want_hash=True, compact=True,
                  want_filter=False) -> DispatchResult:
        torch = self._torch()
        q = torch.empty(max(n, 1), dtype=torch.int16, device=dev)
        h = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if want_hash else None
        qi = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if compact else None
        qs = torch.empty(self.nb_queues + 2, dtype=torch.int32, device=dev) if compact else None
        f = torch.empty(max(n, 1), dtype=torch.int8, device=dev) if want_filter else None
        return DispatchResult(q, h, qi, qs, f)

    def synth(self, profile: int, n: int, first: int = 0, seed: int = 0x9E3779B97F4A7C15,
              nflows: int = 1 << 20, stride: int = abi.WIN_MIN, stream=None):
        """Synthetic header windows + data_len written straight into HBM."""
        torch = self._torch()
        dev = torch.device("cuda", self.device)
        win = torch.empty(max(n, 1) * stride, dtype=torch.uint8, device=dev)
        lens = torch.empty(max(n, 1), dtype=torch.int16, device=dev)
        p = abi.SynthParams(seed & 0xFFFFFFFFFFFFFFFF, profile, nflows)
        rc = self._lib.yrss_synth_dev(self._ctx, ctypes.byref(p), first, n, _ptr(win), stride,
                                      _ptr(lens), self._stream(stream))
        abi.check(rc, "yrss_synth_dev")
        return win, lens[:n] if n else lens[:0]

    # -- host-resident paths (synchronous) ----------------------------------
    def dispatch_frames(self, frames, want_hash=True, compact=True) -> DispatchResult:
        """Classify a list of frames (bytes) — one toeplitz_dispatch per frame."""
        n = len(frames)
        bufs = [np.frombuffer(bytes(f), dtype=np.uint8) if len(f) else np.zeros(1, np.uint8)
                for f in frames]
        ptrs = np.array([b.ctypes.data for b in bufs], dtype=np.uint64)
        lens = np.array([len(f) for f in frames], dtype=np.uint16)
        if np.any(lens != np.array([len(f) for f in frames])):
            raise ValueError("frame longer than 65535 bytes")
        q = np.empty(max(n, 1), np.int16)
        h = np.empty(max(n, 1), np.uint32) if want_hash else None
        qi = np.empty(max(n, 1), np.uint32) if compact else None
        qs = np.empty(self.nb_queues + 2, np.uint32) if compact else None
        rc = self._lib.yrss_dispatch_frames(self._ctx, _ptr(ptrs), _ptr(lens), n, _ptr(q),
                                            _ptr(h), _ptr(qi), _ptr(qs))
        abi.check(rc, "yrss_dispatch_frames")
        return DispatchResult(q[:n], None if h is None else h[:n],
                              None if qi is None else qi[:n], qs)

    def dispatch_burst(self, mbuf_ptrs: np.ndarray, want_hash=True, compact=True,
                       write_rss=False, async_=False) -> DispatchResult:
        """Classify a burst of ``struct rte_mbuf *`` (uint64 addresses).

        ``async_=True`` (YRSS_F_ASYNC) returns once the burst is queued; the
        result's arrays are valid after :meth:`wait`."""
        mb = np.ascontiguousarray(mbuf_ptrs, dtype=np.uint64)
        n = int(mb.size)
        q = np.empty(max(n, 1), np.int16)
        h = np.empty(max(n, 1), np.uint32) if want_hash else None
        qi = np.empty(max(n, 1), np.uint32) if compact else None
        qs = np.empty(self.nb_queues + 2, np.uint32) if compact else None
        flags = (abi.F_WRITE_RSS if write_rss else 0) | (abi.F_ASYNC if async_ else 0)
        rc = self._lib.yrss_dispatch_burst(self._ctx, _ptr(mb), n, _ptr(q), _ptr(h), _ptr(qi),
                                           _ptr(qs), flags)
        abi.check(rc, "yrss_dispatch_burst")
        self._inflight = mb if async_ else None   # keep the pointer array alive
        return DispatchResult(q[:n], None if h is None else h[:n],
                              None if qi is None else qi[:n], qs)

    def wait(self) -> None:
        """Complete the burst queued with ``async_=True`` (``yrss_wait``)."""
        rc = self._lib.yrss_wait(self._ctx)
        self._inflight = None
        self._ck(rc, "yrss_wait")

    # -- persistent burst worker ------------------------------------------------
    def worker_start(self, nslots: int = 16, nblocks: int = 4) -> None:
        """Start the persistent small-burst worker (``yrss_worker_start``)."""
        abi.check(self._lib.yrss_worker_start(self._ctx, nslots, nblocks), "yrss_worker_start")
        self._wk = {}

    def worker_submit(self, mbuf_ptrs: np.ndarray, want_hash=True, compact=True,
                      write_rss=False) -> int:
        """Queue one burst of ``struct rte_mbuf *`` (registered memory); returns
        its ticket.  :meth:`worker_poll` returns the DispatchResult."""
        mb = np.ascontiguousarray(mbuf_ptrs, dtype=np.uint64)
        n = int(mb.size)
        q = np.empty(max(n, 1), np.int16)
        h = np.empty(max(n, 1), np.uint32) if want_hash else None
        qi = np.empty(max(n, 1), np.uint32) if compact else None
        qs = np.empty(self.nb_queues + 2, np.uint32) if compact else None
        t = ctypes.c_uint64()
        rc = self._lib.yrss_worker_submit(self._ctx, _ptr(mb), n, _ptr(q), _ptr(h), _ptr(qi),
                                          _ptr(qs), abi.F_WRITE_RSS if write_rss else 0,
                                          ctypes.byref(t))
        abi.check(rc, "yrss_worker_submit")
        self._wk[t.value] = DispatchResult(q[:n], None if h is None else h[:n],
                                           None if qi is None else qi[:n], qs)
        return t.value

    def worker_submit_frames(self, data_ptrs: np.ndarray, lens: np.ndarray, want_hash=True,
                             compact=True) -> int:
        """Queue one burst of (frame data pointer, data_len) pairs in registered
        memory (``yrss_worker_submit_frames``); returns its ticket."""
        dp = np.ascontiguousarray(data_ptrs, dtype=np.uint64)
        ln = np.ascontiguousarray(lens, dtype=np.uint16)
        n = int(dp.size)
        if ln.size != n:
            raise ValueError("data_ptrs and lens differ in length")
        q = np.empty(max(n, 1), np.int16)
        h = np.empty(max(n, 1), np.uint32) if want_hash else None
        qi = np.empty(max(n, 1), np.uint32) if compact else None
        qs = np.empty(self.nb_queues + 2, np.uint32) if compact else None
        t = ctypes.c_uint64()
        rc = self._lib.yrss_worker_submit_frames(self._ctx, _ptr(dp), _ptr(ln), n, _ptr(q),
                                                 _ptr(h), _ptr(qi), _ptr(qs), ctypes.byref(t))
        abi.check(rc, "yrss_worker_submit_frames")
        self._wk[t.value] = DispatchResult(q[:n], None if h is None else h[:n],
                                           None if qi is None else qi[:n], qs)
        return t.value

    def worker_submit_windows(self, win: np.ndarray, stride: int, lens: np.ndarray,
                              want_hash=True, compact=True) -> int:
        """Queue one burst of contiguous windows (window i at win[i * stride:])
        that lie in registered memory (``yrss_worker_submit_windows``)."""
        ln = np.ascontiguousarray(lens, dtype=np.uint16)
        n = int(ln.size)
        q = np.empty(max(n, 1), np.int16)
        h = np.empty(max(n, 1), np.uint32) if want_hash else None
        qi = np.empty(max(n, 1), np.uint32) if compact else None
        qs = np.empty(self.nb_queues + 2, np.uint32) if compact else None
        t = ctypes.c_uint64()
        rc = self._lib.yrss_worker_submit_windows(self._ctx, _ptr(win), stride, _ptr(ln), n,
                                                  _ptr(q), _ptr(h), _ptr(qi), _ptr(qs),
                                                  ctypes.byref(t))
        abi.check(rc, "yrss_worker_submit_windows")
        self._wk[t.value] = DispatchResult(q[:n], None if h is None else h[:n],
                                           None if qi is None else qi[:n], qs)
        return t.value

    def toeplitz_dispatch(self, frame: bytes, queue_id: int = 0) -> int:
        """The per-packet registration shim (``yrss_toeplitz_dispatch``) on this
        context: ``toeplitz_dispatch``'s return value for one frame, computed on
        the GPU.  One launch per call: for compatibility, not speed."""
        abi.check(self._lib.yrss_set_dispatch_ctx(self._ctx), "yrss_set_dispatch_ctx")
        buf = ctypes.create_string_buffer(bytes(frame), len(frame))
        return int(self._lib.yrss_toeplitz_dispatch(ctypes.cast(buf, ctypes.c_void_p),
                                                    len(frame), queue_id, self.nb_queues))

    def worker_poll(self, ticket: int, wait: bool = True):
        """The burst's DispatchResult, or None while it is pending (wait=False)."""
        rc = self._lib.yrss_worker_poll(self._ctx, ticket, 1 if wait else 0)
        if rc == -11:   # -EAGAIN
            return None
        res = self._wk.pop(ticket, None)
        self._ck(rc, "yrss_worker_poll")
        return res

    def worker_stop(self) -> None:
        abi.check(self._lib.yrss_worker_stop(self._ctx), "yrss_worker_stop")
        self._wk = {}

    def register_host_memory(self, base: int, nbytes: int) -> None:
        abi.check(self._lib.yrss_register_host_memory(self._ctx, base, nbytes),
                  "yrss_register_host_memory")

    def unregister_host_memory(self, base: int) -> None:
        abi.check(self._lib.yrss_unregister_host_memory(self._ctx, base),
                  "yrss_unregister_host_memory")

    def dispatch_burst_zc(self, mbuf_ptrs: np.ndarray, want_hash=True, compact=True,
                          write_rss=False, async_=False) -> DispatchResult:
        """Zero-copy burst: mbufs in registered host memory are read by the GPU.
        ``async_`` as in :meth:`dispatch_burst`."""
        mb = np.ascontiguousarray(mbuf_ptrs, dtype=np.uint64)
        n = int(mb.size)
        q = np.empty(max(n, 1), np.int16)
        h = np.empty(max(n, 1), np.uint32) if want_hash else None
        qi = np.empty(max(n, 1), np.uint32) if compact else None
        qs = np.empty(self.nb_queues + 2, np.uint32) if compact else None
        flags = (abi.F_WRITE_RSS if write_rss else 0) | (abi.F_ASYNC if async_ else 0)
        rc = self._lib.yrss_dispatch_burst_zc(self._ctx, _ptr(mb), n, _ptr(q), _ptr(h), _ptr(qi),
                                              _ptr(qs), flags)
        abi.check(rc, "yrss_dispatch_burst_zc")
        self._inflight = mb if async_ else None
        return DispatchResult(q[:n], None if h is None else h[:n],
                              None if qi is None else qi[:n], qs)

    def route_burst(self, mbuf_ptrs: np.ndarray, queue_id: int, enqueue, clone, release,
                    kni_primary: bool = True):
        """process_packets' hand-off for a burst (``yrss_route_burst``).

        ``enqueue(queue, [mbuf addr...]) -> n_enqueued``, ``clone(mbuf, queue)
        -> addr or 0``, ``release(mbuf)`` are called back from C.  Returns
        (local list, kni list, RouteResult)."""
        mb = np.ascontiguousarray(mbuf_ptrs, dtype=np.uint64)
        n = int(mb.size)

        def _enq(user, queue, objs, cnt):
            return int(enqueue(int(queue), [int(objs[i] or 0) for i in range(cnt)]))

        def _clone(user, m, queue):
            return int(clone(int(m or 0), int(queue)) or 0)

        def _rel(user, m):
            release(int(m or 0))

        ops = abi.RouteOps(abi.ENQUEUE_FN(_enq), abi.CLONE_FN(_clone), abi.RELEASE_FN(_rel), None)
        local = np.zeros(max(n, 1), np.uint64)
        kni = np.zeros(max(2 * n, 1), np.uint64)
        res = abi.RouteResult()
        rc = self._lib.yrss_route_burst(self._ctx, _ptr(mb), n, queue_id, 1 if kni_primary else 0,
                                        ctypes.byref(ops), _ptr(local), _ptr(kni),
                                        ctypes.byref(res))
        abi.check(rc, "yrss_route_burst")
        return local[:res.n_local].tolist(), kni[:res.n_kni].tolist(), res

    # -- connect-side RSS check (ff_rss_check) -------------------------------
    def rss_check_dev(self, tuples, nb_queues: int, reta_size: int, queueid: int, stream=None):
        """ff_rss_check for n raw 12-byte tuples on the device (uint8 tensor n*12).
        Returns (ok uint8 tensor, hash int32 tensor)."""
        torch = self._torch()
        n = int(tuples.numel()) // 12
        ok = torch.empty(max(n, 1), dtype=torch.uint8, device=tuples.device)
        h = torch.empty(max(n, 1), dtype=torch.int32, device=tuples.device)
        abi.check(self._lib.yrss_rss_check_dev(self._ctx, _ptr(tuples), n, nb_queues, reta_size,
                                               queueid, _ptr(ok), _ptr(h), self._stream(stream)),
                  "yrss_rss_check_dev")
        return ok[:n], h[:n]

    def rss_lport_sweep(self, faddr: int, laddr: int, fport: int, nb_queues: int,
                        reta_size: int, queueid: int) -> np.ndarray:
        """Bitmap (2048 uint32) of every stored lport value accepted by ff_rss_check."""
        bm = np.zeros(2048, np.uint32)
        abi.check(self._lib.yrss_rss_lport_sweep(self._ctx, faddr, laddr, fport, nb_queues,
                                                 reta_size, queueid, _ptr(bm)),
                  "yrss_rss_lport_sweep")
        return bm

    # -- timing hook --------------------------------------------------------
    def timing_enable(self, mask: int = 1 << abi.K_PARSE_HASH) -> None:
        """Bracket every launch of kernel k (bit k of mask, abi.K_*) with HIP
        events on its own dispatch packet; 0 disables."""
        abi.check(self._lib.yrss_timing_enable(self._ctx, int(mask)), "yrss_timing_enable")

    def timing_read(self, kernel: int) -> tuple[float, int]:
        ms = ctypes.c_double()
        cnt = ctypes.c_uint32()
        abi.check(self._lib.yrss_timing_read(self._ctx, kernel, ctypes.byref(ms),
                                             ctypes.byref(cnt)), "yrss_timing_read")
        return ms.value, cnt.value

    def timing_quantile(self, kernel: int, q: float = 0.5) -> float:
        """q-quantile of kernel's per-launch durations (ms) since timing_enable."""
        ms = ctypes.c_double()
        abi.check(self._lib.yrss_timing_quantile(self._ctx, kernel, q, ctypes.byref(ms)),
                  "yrss_timing_quantile")
        return ms.value

    def status(self) -> int:
        """Synchronise and return (then clear) the device-side fault state:
        0, or -EIO if a list guard fired (yrss_status; details: fault_info)."""
        return int(self._lib.yrss_status(self._ctx))

    def fault_info(self):
        """Synchronise and return (then clear) the fault record as
        (code, kernel, where, value); code 0 (abi.FAULT_NONE) = no guard fired."""
        f = abi.Fault()
        abi.check(self._lib.yrss_fault_info(self._ctx, ctypes.byref(f)), "yrss_fault_info")
        return (int(f.code), int(f.kernel), int(f.where), int(f.value))

    def set_tuning(self, chunk_tiles: int = 0, span_tiles: int = 0, parse_blocks: int = 0,
                   one_launch: int = 0, scatter_xcd: int = -1, scan_kernel: int = 0) -> None:
        """Layout overrides for tests and measurements (yrss_set_tuning); the
        results never depend on them."""
        t = abi.Tuning(chunk_tiles, span_tiles, parse_blocks, one_launch, scatter_xcd, scan_kernel)
        abi.check(self._lib.yrss_set_tuning(self._ctx, ctypes.byref(t)), "yrss_set_tuning")

    def grid_for(self, n: int) -> int:
        return int(self._lib.yrss_grid_for(self._ctx, n))


class FanOut:
    """One dispatcher thread's host bursts spread round-robin over several
    contexts / GPUs (``yrss_fanout_*``), returned in submission order by
    :meth:`next` so per-queue FIFO holds over the whole stream."""

    def __init__(self, devices, nb_procs: int = 3, nb_queues: int | None = None,
                 soft_dispatch: int = 1, dispatch_only_core: int = 1, nslots: int = 16,
                 nblocks: int = 4):
        self._lib = abi.load()
        cfg = abi.default_config()
        cfg.nb_procs = nb_procs
        cfg.nb_queues = nb_procs if nb_queues is None else nb_queues
        cfg.soft_dispatch = soft_dispatch
        cfg.dispatch_only_core = dispatch_only_core
        self.nb_queues = int(cfg.nb_queues)
        devs = (ctypes.c_int * len(devices))(*devices)
        f = ctypes.c_void_p()
        abi.check(self._lib.yrss_fanout_init(ctypes.byref(cfg), devs, len(devices), nslots,
                                             nblocks, ctypes.byref(f)), "yrss_fanout_init")
        self._f = f
        self._res = {}

    def close(self) -> None:
        if getattr(self, "_f", None) and self._f.value:
            rc = self._lib.yrss_fanout_fini(self._f)
            self._f = ctypes.c_void_p()
            abi.check(rc, "yrss_fanout_fini")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def register_host_memory(self, base: int, nbytes: int) -> None:
        abi.check(self._lib.yrss_fanout_register_host_memory(self._f, base, nbytes),
                  "yrss_fanout_register_host_memory")

    def unregister_host_memory(self, base: int) -> None:
        abi.check(self._lib.yrss_fanout_unregister_host_memory(self._f, base),
                  "yrss_fanout_unregister_host_memory")

    def _outs(self, n):
        q = np.empty(max(n, 1), np.int16)
        h = np.empty(max(n, 1), np.uint32)
        qi = np.empty(max(n, 1), np.uint32)
        qs = np.empty(self.nb_queues + 2, np.uint32)
        return q, h, qi, qs

    def submit(self, mbuf_ptrs: np.ndarray) -> int:
        mb = np.ascontiguousarray(mbuf_ptrs, dtype=np.uint64)
        n = int(mb.size)
        q, h, qi, qs = self._outs(n)
        t = ctypes.c_uint64()
        abi.check(self._lib.yrss_fanout_submit(self._f, _ptr(mb), n, _ptr(q), _ptr(h), _ptr(qi),
                                               _ptr(qs), 0, ctypes.byref(t)), "yrss_fanout_submit")
        self._res[t.value] = DispatchResult(q[:n], h[:n], qi[:n], qs)
        return t.value

    def submit_frames(self, data_ptrs: np.ndarray, lens: np.ndarray) -> int:
        dp = np.ascontiguousarray(data_ptrs, dtype=np.uint64)
        ln = np.ascontiguousarray(lens, dtype=np.uint16)
        n = int(dp.size)
        q, h, qi, qs = self._outs(n)
        t = ctypes.c_uint64()
        abi.check(self._lib.yrss_fanout_submit_frames(self._f, _ptr(dp), _ptr(ln), n, _ptr(q),
                                                      _ptr(h), _ptr(qi), _ptr(qs),
                                                      ctypes.byref(t)),
                  "yrss_fanout_submit_frames")
        self._res[t.value] = DispatchResult(q[:n], h[:n], qi[:n], qs)
        return t.value

    def next(self, wait: bool = True):
        """(ticket, DispatchResult) of the oldest outstanding burst once done;
        None while it runs (wait=False) or when nothing is outstanding."""
        t = ctypes.c_uint64()
        rc = self._lib.yrss_fanout_next(self._f, 1 if wait else 0, ctypes.byref(t))
        if rc in (-11, -2):   # -EAGAIN, -ENOENT
            return None
        res = self._res.pop(t.value, None) if rc in (0, -14) else None
        abi.check(rc, "yrss_fanout_next")
        return t.value, res
