#!/usr/bin/env python3
"""A/B of the windows form's dispatcher copy (tools/yrss_cbench, worker form
2): plain memcpy into the registered staging against non-temporal 16-byte
stores (YRSS_CBENCH_WIN_NT=1), alternated, on the CPU bench.py pins the
dispatcher to (gpu_placement: a physical core of the GPU's node).

    python tools/win_ab.py [--rounds 3] [--bursts 32,1024]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--bursts", default="32,1024")
    ap.add_argument("--pools", default=str(1 << 20),
                    help="mbuf pool sizes: 2^20 is cache-cold (2.4 GB); 16384 keeps the touched "
                         "header and window lines LLC-resident, as an rx ring's recycled mbufs")
    args = ap.parse_args()
    place = bench.gpu_placement(bench.device_identity(0, False))
    print(json.dumps({"placement": place}), flush=True)
    exe = ROOT / "tools" / "yrss_cbench"
    for pool, burst in ((int(p), int(b)) for p in args.pools.split(",")
                        for b in args.bursts.split(",")):
        blocks = 128 if burst <= 64 else 32
        for r in range(args.rounds):
            for nt in ("0", "1"):
                env = {**os.environ, "YRSS_CBENCH_MODES": "4", "YRSS_CBENCH_REPEAT": "1",
                       "YRSS_CBENCH_WORKER_DEPTH": str(4 * blocks),
                       "YRSS_CBENCH_WORKER_BLOCKS": str(blocks),
                       "YRSS_CBENCH_WORKER_SLOTOUT": "1", "YRSS_CBENCH_WORKER_FRAMES": "2",
                       "YRSS_CBENCH_WIN_NT": nt}
                if place.get("dispatch_cpu") is not None:
                    env["YRSS_CBENCH_CPU"] = str(place["dispatch_cpu"])
                out = subprocess.run([str(exe), "1", str(pool), str(burst), "1"],
                                     capture_output=True, text=True, timeout=240, env=env)
                for line in out.stdout.splitlines():
                    try:
                        d = json.loads(line)
                    except ValueError:
                        continue
                    print(json.dumps({"pool": pool, "burst": burst, "round": r, "win_nt": int(nt),
                                      "mpps": d["mpps"], "submit_cycles": d.get("submit_cycles"),
                                      "poll_cycles": d.get("poll_cycles"), "cpu": d.get("cpu")}),
                          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
