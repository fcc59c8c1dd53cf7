#!/usr/bin/env python3
"""Host placement of the host-resident worker rows: the GPU's NUMA node,
the CPUs this job may use per node, the cgroup CPU quota, then the 32-packet
worker (frames form, 128 workgroups) with the dispatcher thread pinned to a
CPU on the GPU's node and to a CPU on every other node the job may use
(tools/yrss_cbench, YRSS_CBENCH_REPEAT runs each).  The pool is first touched
by the pinned thread, so it lands on that CPU's node.

    python tools/numa_probe.py [--repeat 3] [--frames 1] [--burst 32] [--load K]

--load K also runs the near-node case with K busy-loop processes pinned to
other CPUs the job may use (the job's cgroup CPU quota then throttles every
thread of the job, the dispatcher included, when the quota is exceeded).
"""
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
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--frames", default="1")
    ap.add_argument("--burst", type=int, default=32)
    ap.add_argument("--blocks", type=int, default=128)
    ap.add_argument("--load", type=int, default=0)
    args = ap.parse_args()
    import torch

    dev = bench.device_identity(0, False)     # device_count/properties: no GPU context
    place = bench.gpu_placement(dev)
    allowed = sorted(os.sched_getaffinity(0))
    nodes = {}
    for nd in sorted(Path("/sys/devices/system/node").glob("node[0-9]*")):
        cpus = [c for c in bench._cpulist((nd / "cpulist").read_text()) if c in set(allowed)]
        if cpus:
            nodes[int(nd.name[4:])] = cpus
    print(json.dumps({"gpu": dev, "placement": place, "quota": bench.cpu_quota(),
                      "allowed": len(allowed),
                      "nodes": {k: f"{v[0]}..{v[-1]} ({len(v)})" for k, v in nodes.items()}}),
          flush=True)
    exe = ROOT / "tools" / "yrss_cbench"
    cases = [(nd, cpus[len(cpus) // 2], 0) for nd, cpus in nodes.items()]
    if args.load and place["gpu_node"] in nodes:
        cpus = nodes[place["gpu_node"]]
        cases.append((place["gpu_node"], cpus[len(cpus) // 2], args.load))
    for nd, cpu, load in cases:
        hogs = []
        others = [c for c in allowed if c != cpu][:load]
        for c in others:
            hogs.append(subprocess.Popen([sys.executable, "-c",
                                          f"import os; os.sched_setaffinity(0, {{{c}}})\nwhile True: pass"]))
        try:
            r = subprocess.run([str(exe), "1", str(1 << 20), str(args.burst), "1"],
                               capture_output=True, text=True, timeout=300,
                               env={**os.environ, "YRSS_CBENCH_MODES": "4",
                                    "YRSS_CBENCH_CPU": str(cpu),
                                    "YRSS_CBENCH_REPEAT": str(args.repeat),
                                    "YRSS_CBENCH_WORKER_DEPTH": str(4 * args.blocks),
                                    "YRSS_CBENCH_WORKER_BLOCKS": str(args.blocks),
                                    "YRSS_CBENCH_WORKER_SLOTOUT": "1",
                                    "YRSS_CBENCH_WORKER_FRAMES": args.frames})
        finally:
            for h in hogs:
                h.kill()
                h.wait()
        for line in r.stdout.splitlines():
            try:
                d = json.loads(line)
            except ValueError:
                continue
            print(json.dumps({"pin_node": nd, "busy_procs": load, "gpu_node": place["gpu_node"], "cpu": d.get("cpu"),
                              "cpu_node": d.get("cpu_node"), "pool_node": d.get("pool_node"),
                              "api": d["api"], "burst": d["burst"], "mpps": d["mpps"],
                              "poll_cycles": d.get("poll_cycles"),
                              "submit_cycles": d.get("submit_cycles")}), flush=True)
        if r.returncode:
            print(r.stderr[-2000:], flush=True)
            return r.returncode
    del torch
    return 0


if __name__ == "__main__":
    sys.exit(main())
