"""Is the parse kernel's floor set by mixing reads and writes?  Times the
ideal-traffic twin (tools/yrss_probe.hip) mixed, reads only and writes only
over 2^24 packets (64-byte windows) and prints the three durations.  Each
mode runs in its own process (the mode is read once per process)."""
import json
import os
import subprocess
import sys

N = 1 << 24


def child(mode: int) -> None:
    import ctypes

    import torch

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = ctypes.CDLL(os.path.join(root, "tools", "libyrss_probe.so"))
    fn = lib.yrss_probe_traffic_launch
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    win = torch.randint(0, 255, (N * 64,), dtype=torch.uint8, device=dev)
    lens = torch.full((N,), 64, dtype=torch.int16, device=dev)
    q = torch.empty(N, dtype=torch.int16, device=dev)
    h = torch.empty(N, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    args = (win.data_ptr(), lens.data_ptr(), q.data_ptr(), h.data_ptr(), N, s.cuda_stream)
    for _ in range(5):
        assert fn(*args) == 0
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    steps = 50
    ev[0].record(s)
    for _ in range(steps):
        fn(*args)
    ev[1].record(s)
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) / steps * 1e3
    nbytes = {0: 72, 1: 66, 2: 6, 3: 6}[mode] * N
    print(json.dumps({"mode": mode, "us": round(us, 1), "TB/s": round(nbytes / us / 1e6, 3)}))
    if mode == 0:   # chip write ceiling for the same 6 B/pkt: torch fills
        ev[0].record(s)
        for _ in range(steps):
            q.fill_(1)
            h.fill_(1)
        ev[1].record(s)
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) / steps * 1e3
        print(json.dumps({"mode": "fill", "us": round(us, 1), "TB/s": round(6 * N / us / 1e6, 3)}),
              file=sys.stderr)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child(int(sys.argv[1]))
        sys.exit(0)
    rows = []
    for mode in (0, 1, 2, 3):
        r = subprocess.run([sys.executable, __file__, str(mode)], capture_output=True, text=True,
                           timeout=180, env={**os.environ, "YRSS_PROBE_MODE": str(mode)})
        if r.returncode:
            print(r.stdout, r.stderr)
            sys.exit(r.returncode)
        rows.append(json.loads(r.stdout.strip().splitlines()[-1]))
        print(json.dumps(rows[-1]))
        if r.stderr.strip():
            print(r.stderr.strip().splitlines()[-1])
    mix, rd, wr, _ = (x["us"] for x in rows)
    print(f"mixed {mix} us; reads only {rd} + writes only {wr} = {rd + wr:.1f} us")
