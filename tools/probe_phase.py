"""Write-phase experiment on the ideal-traffic twin (tools/yrss_probe.hip,
yrss_probe_phase): the parse kernel's traffic with each wave's outputs held in
LDS and written when its buffer fills (cap chunks) or when the chip-wide clock
enters a new period, against the plain twin (mode 0) and its reads alone
(mode 1).  Same four rotated 2^24-packet batches as bench.py.

    python tools/probe_phase.py
"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch

    from yastack_amd import SoftRss, abi

    n, stride = 1 << 24, 64
    lib = ctypes.CDLL(str(ROOT / "tools" / "libyrss_probe.so"))
    mode_fn = lib.yrss_probe_traffic_launch_mode
    mode_fn.restype = ctypes.c_int
    mode_fn.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
    ph = lib.yrss_probe_phase_launch
    ph.restype = ctypes.c_int
    ph.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_uint32, ctypes.c_uint32]
    eng = SoftRss(3, 3, 1, 1, device=0, max_burst=0)
    bufs = []
    for k in range(4):
        w, ln = eng.synth(abi.SYN_UDP4, n, k * n, stride=stride)
        o = eng.alloc_out(n, w.device, want_hash=True, compact=False)
        bufs.append((w, ln, o))
    stream = torch.cuda.current_stream()

    def timed(call, steps=40):
        for i in range(4):
            call(bufs[i % 4])
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for i in range(steps):
            call(bufs[i % 4])
        ev[1].record(stream)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / steps * 1e3

    def a(b):
        w, ln, o = b
        return (w.data_ptr(), ln.data_ptr(), o.q.data_ptr(), o.hash.data_ptr(), n,
                stream.cuda_stream)

    rows = [("twin (mode 0)", lambda b: mode_fn(*a(b), 0)),
            ("reads only (mode 1)", lambda b: mode_fn(*a(b), 1)),
            ("outputs in the window records (mode 5)", lambda b: mode_fn(*a(b), 5))]
    for cap in (() if "--rows" in sys.argv else (1, 2, 4)):
        rows.append((f"buffer {cap} chunks, no clock", lambda b, cap=cap: ph(*a(b), 0, 1, cap)))
    for period in (() if "--rows" in sys.argv else (100, 200, 500, 1000)):
        rows.append((f"buffer 4 chunks, clock period {period * 10} ns",
                     lambda b, p=period: ph(*a(b), 1, p, 4)))
    for rep in range(2):
        for name, call in rows:
            us = timed(call)
            print(f"r{rep + 1} {name}: {us:.2f} us = {72 * n / us / 1e6:.2f} TB/s (72 B/pkt)",
                  flush=True)
    eng.close()


if __name__ == "__main__":
    main()
