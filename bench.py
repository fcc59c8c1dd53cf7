#!/usr/bin/env python3
"""bench.py — device-resident soft-RSS parse+hash throughput (BASELINE.json).

One "step" = one full soft-RSS pass over one batch resident in HBM: parse +
Toeplitz hash + queue for every packet (toeplitz_dispatch,
fs/lib/ff_dpdk_if.c:1945-2113) plus the per-queue FIFO index lists that stand
in for process_packets' enqueue into dispatch_ring[port][q] (:1078-1094).

Workload (BASELINE.json configs[1]): 64 B Eth/IPv4/UDP, 1M random 5-tuples,
2^24 packets per GPU generated on-device, 64-byte windows + data_len;
fs/config/config.ini knobs (nb_procs 3, soft_dispatch 1, dispatch_only_core 1).

Multi-GPU: one process per GPU (torchrun), each rank classifies its own
contiguous shard of the global packet stream — no collective on the data path
(SURVEY.md §8(e)); gloo carries only the barrier and the max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--profile udp4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PCIE_GEN5_X16_GBS = 64.0  # one direction of the host link, GB/s
PROFILES = {"udp4_1flow": 0, "udp4": 1, "imix": 2, "vlan6_tcp": 3, "jumbo_tcp4": 4,
            "tcp4": 5, "fuzz": 6}
WORKLOADS = {
    "udp4": "64B UDP/IPv4, 1M random 5-tuples (BASELINE configs[1])",
    "imix": "IMIX 64/570/1500 7:4:1 TCP+UDP/IPv4, 1M flows (configs[2])",
    "vlan6_tcp": "64B VLAN+IPv6+TCP, 4M flows (configs[3])",
    "jumbo_tcp4": "9000B jumbo TCP/IPv4 header-bound, 16M flows (configs[4])",
    "tcp4": "64B TCP/IPv4, 1M flows (hash path on every packet)",
    "udp4_1flow": "64B UDP/IPv4 single flow (configs[0] traffic)",
    "fuzz": "adversarial headers",
}
NFLOWS = {"udp4": 1 << 20, "imix": 1 << 20, "vlan6_tcp": 1 << 22, "jumbo_tcp4": 1 << 24,
          "tcp4": 1 << 20, "udp4_1flow": 1, "fuzz": 1}
SEED = 0x9E3779B97F4A7C15


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--profile", default="udp4", choices=sorted(PROFILES))
    ap.add_argument("--pkts", type=int, default=1 << 24, help="packets per GPU")
    ap.add_argument("--stride", type=int, default=64)
    ap.add_argument("--batches", type=int, default=4,
                    help="distinct batches rotated step by step: a batch re-read every "
                         "step keeps part of itself in the 256 MB MALL (~8%% faster), "
                         "which a stream of new packets would not")
    ap.add_argument("--nb-procs", type=int, default=3)
    ap.add_argument("--nb-queues", type=int, default=None)
    ap.add_argument("--dispatch-only-core", type=int, default=1)
    ap.add_argument("--no-compact", action="store_true",
                    help="parse+hash only (no per-queue lists)")
    ap.add_argument("--filter", action="store_true",
                    help="also run the fused KNI protocol_filter (1 B/pkt more)")
    ap.add_argument("--cpu-seconds", type=float, default=16.0,
                    help="target CPU-baseline duration over its 8 cells (0 disables)")
    ap.add_argument("--pcie", type=int, default=1,
                    help="also time the host-resident (PCIe-inclusive) paths with "
                         "tools/yrss_cbench at N=1 (reported beside value, never as value)")
    ap.add_argument("--check", type=int, default=1 << 20,
                    help="packets verified against the oracle after timing (0 = off)")
    ap.add_argument("--kernel-timing", type=int, default=1,
                    help="time the parse kernel with HIP events inside the timed region "
                         "(0: diagnosis only, roofline.achieved is then null)")
    ap.add_argument("--pmc", default=str(ROOT / "profiles" / "pmc_parse_hash.json"),
                    help="rocprofv3 PMC summary used for roofline.traffic")
    ap.add_argument("--tune", default="",
                    help="layout overrides for measurements, k=v[,k=v] (yrss_set_tuning "
                         "fields: chunk_tiles, span_tiles, parse_blocks, scatter_xcd, scan_kernel)")
    ap.add_argument("--extra-configs", default="imix,vlan6_tcp,jumbo_tcp4",
                    help="after the headline, each rank also classifies a --pkts shard of "
                         "these profiles (BASELINE configs[2] IMIX, configs[3] and configs[4], "
                         "the 8-GPU configs), reported under configs_extra, never as value "
                         "('' = off)")
    ap.add_argument("--test-hooks", default="",
                    help="measurements only: run libyrss_test.so with its yrss_debug_* hooks, "
                         "k=v[,k=v] (merge, groups); the line says so")
    ap.add_argument("--dry", action="store_true",
                    help="plumbing check without a GPU (rank spawn, barrier, reductions); "
                         "prints a line marked dry, never a measurement")
    return ap.parse_args(argv)


# ---- distributed plumbing (gloo: control only) -----------------------------------
def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv) -> int:
    """`python bench.py --gpus N` without a launcher: start N fresh rank
    processes (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their env) and return
    the worst exit status.  The parent never touches the GPU: each child picks
    its device from LOCAL_RANK before any HIP call.  If one rank fails, the
    others are stopped (they would wait at the barrier)."""
    import subprocess

    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = {**os.environ, "RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
               "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": port}
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *argv],
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            s = p.poll()
            if s is None:
                continue
            live.remove(p)
            if s != 0:
                rc = rc or (s if s > 0 else 128 - s)
                for q in live:
                    q.terminate()
        if live:
            time.sleep(0.05)
    return rc


def dist_setup(gpus: int):
    """World size from the launcher's env (torchrun); it must agree with
    --gpus.  Fails loudly instead of silently measuring fewer GPUs."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}; "
                         "launch with --gpus equal to the rank count")
    if os.environ.get("YRSS_BENCH_ONE_DEVICE"):
        local = 0            # rehearsal of the N>1 path on a single GPU
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return world, rank, local


def device_identity(local: int, dry: bool) -> str:
    """PCI location (domain:bus:device) of the GPU this rank drives."""
    if dry:    # the test hook stands in for two ranks opening one device
        return "dry-device" if os.environ.get("YRSS_BENCH_FAKE_SAME_DEVICE") \
            else f"dry-rank-local{local}"
    import torch

    p = torch.cuda.get_device_properties(local)
    dom = getattr(p, "pci_domain_id", 0)
    bus = getattr(p, "pci_bus_id", None)
    dev = getattr(p, "pci_device_id", None)
    if bus is None:
        return f"{p.name}#{local}"
    return f"{dom:04x}:{bus:02x}:{dev:02x}"


def gather_objects(obj, world: int):
    if world == 1:
        return [obj]
    import torch.distributed as dist

    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


# ---- CPU baseline (oracle, rank 0) -------------------------------------------------
CPU_PROFILES = ("udp4", "tcp4")        # the headline stream, and every packet hashed
CPU_VARIANTS = ("bit_serial", "table")  # toeplitz_hash as written; 12x256 byte tables
CPU_RUNS = 3                            # timed windows per cell: median, min, max
OVERLAP_MIN = 0.95                      # a multi-process cell below this is flagged
# packets a process re-runs: 4 MiB of windows, LLC-resident as an rx burst's headers
# are after DDIO (8 processes share a CCD's 32 MB L3).  2^20 packets (64 MiB) made
# the udp4 cells a test of one core's DRAM streaming rate: 1-core medians of
# 224-533 Mpkt/s across boxes for the same code.
CPU_SAMPLE_PKTS = 1 << 16


def cpu_worker(spec: str) -> int:
    """One pinned CPU-baseline process (bench.py --cpu-worker prof:variant:cpu):
    the oracle's toeplitz_dispatch restatement over CPU_SAMPLE_PKTS packets of the stream,
    one call per packet, inlined or (variant suffix "_fnptr") through the
    registered-dispatcher function pointer as process_packets calls it
    (ff_dpdk_if.c:1078-1079).  Every "go START END" line on stdin runs one
    window between those CLOCK_MONOTONIC instants (ns), so all processes of a
    cell run over the same stretch of time; the answer carries the packets and
    the window's actual first and last instants."""
    prof, variant, cpu = spec.split(":")
    if cpu != "-":
        os.sched_setaffinity(0, {int(cpu)})     # what taskset -c does
    from oracle import oracle

    n = CPU_SAMPLE_PKTS
    win, lens = oracle.synth(PROFILES[prof], n, 0, SEED, NFLOWS[prof], 64)
    c = oracle.cfg(3, 3, 1, 1)                  # fs/config/config.ini knobs
    fast = variant.startswith("table")
    fnptr = variant.endswith("_fnptr")
    t = time.monotonic_ns()
    oracle.bench_window(win, 64, lens, c, fast, fnptr, t, t + 20_000_000)   # warm caches
    print("ready", flush=True)
    for line in sys.stdin:
        parts = line.split()
        if not parts or parts[0] != "go":
            break
        pkts, t0, t1 = oracle.bench_window(win, 64, lens, c, fast, fnptr, int(parts[1]),
                                           int(parts[2]))
        print(json.dumps({"pkts": pkts, "t0": t0 / 1e9, "t1": t1 / 1e9}), flush=True)
    return 0


def _cpu_run(prof: str, variant: str, secs: float, cpus, runs: int = CPU_RUNS):
    """len(cpus) pinned worker processes, started once and given `runs`
    common windows [start, start + secs] on CLOCK_MONOTONIC.  A window's rate
    is the sum of the processes' own rates, each over its own actual stretch;
    `overlap` is the shortest common stretch of a window over its longest
    process (1.0 = side by side the whole time; below OVERLAP_MIN the cell is
    flagged, its rate is then not a simultaneous one)."""
    import subprocess
    import statistics

    procs = [subprocess.Popen([sys.executable, str(Path(__file__).resolve()), "--cpu-worker",
                               f"{prof}:{variant}:{cpu}"],
                              stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
             for cpu in cpus]
    rates, overlaps = [], []
    try:
        for p in procs:
            if p.stdout.readline().strip() != "ready":
                raise RuntimeError("cpu worker failed to start")
        for _ in range(runs):
            start = time.monotonic_ns() + 50_000_000    # every process is waiting by then
            end = start + int(secs * 1e9)
            for p in procs:
                p.stdin.write(f"go {start} {end}\n")
                p.stdin.flush()
            res = [json.loads(p.stdout.readline()) for p in procs]
            rates.append(sum(r["pkts"] / (r["t1"] - r["t0"]) for r in res) / 1e6)
            common = min(r["t1"] for r in res) - max(r["t0"] for r in res)
            overlaps.append(max(0.0, common) / max(r["t1"] - r["t0"] for r in res))
        for p in procs:
            p.stdin.write("end\n")
            p.stdin.flush()
    finally:
        for p in procs:
            p.wait(timeout=600)
    out = {"mpps": round(statistics.median(rates), 2), "min": round(min(rates), 2),
           "max": round(max(rates), 2), "runs": len(rates),
           "overlap": round(min(overlaps), 4)}
    if len(cpus) > 1 and out["overlap"] < OVERLAP_MIN:
        out["flag"] = f"overlap {out['overlap']} < {OVERLAP_MIN}: not a simultaneous rate"
    return out


def cpu_quota():
    """CPUs this job may keep busy: the cgroup CPU quota (v2 cpu.max, else v1
    cfs_quota/period), capped by the affinity mask.  (count, source)."""
    allowed = len(os.sched_getaffinity(0))
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = Path(path).read_text().split()[:2]
            if q != "max":
                n = max(1, -(-int(q) // int(per)))
                return min(n, allowed), f"cgroup cpu.max {q} {per}"
        except (OSError, ValueError):
            pass
    try:
        q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        if q > 0:
            return min(allowed, max(1, -(-q // per))), f"cgroup cfs_quota_us {q} / {per}"
    except (OSError, ValueError):
        pass
    return allowed, "no cgroup CPU quota: sched_getaffinity"


def physical_cores(cpus):
    """One logical CPU per physical core (the first SMT sibling), in order."""
    seen, out = set(), []
    for c in cpus:
        try:
            sib = Path(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read_text()
            key = min(_cpulist(sib))
        except (OSError, ValueError):
            key = c
        if key not in seen:
            seen.add(key)
            out.append(c)
    return out


def cpu_baseline(args, nb_queues):
    """the reference's algorithm on the GPU box's host cores.
    Both ports (bit-serial as the reference writes toeplitz_hash, and
    table-driven), on the headline UDP stream and all-TCP, on 1 core (the
    reference's single dispatching lcore, ff_dpdk_if.c:1653) and on one GPU's
    share of the box (16 cores), as independent processes pinned one per
    physical core; and on every core the job's CPU quota lets it keep busy
    (cgroup cpu.max, stated), SURVEY §8(d).  The 1-core cells also run through
    the registered-dispatcher function pointer (`_fnptr`), the call form of
    process_packets (ff_dpdk_if.c:1078-1079).  Every cell is the median of
    CPU_RUNS common timed windows with its min and max.  `value` is the
    bit-serial port on 1 core over the bench's own stream, called through the
    function pointer as the reference calls it; `value_inlined` beside it."""
    allowed = sorted(os.sched_getaffinity(0))
    phys = physical_cores(allowed) or allowed
    quota, qsrc = cpu_quota()
    share_n = max(1, min(16, quota, len(phys)))
    share = phys[:share_n]                          # one GPU's share of the box's cores
    cells = [phys[:1], share]
    profs = list(dict.fromkeys([args.profile, *CPU_PROFILES]))   # the bench's own stream first
    n_cells = len(profs) * (len(cells) * len(CPU_VARIANTS) + len(CPU_VARIANTS)) + 1
    secs = max(0.3, args.cpu_seconds / (n_cells * CPU_RUNS))
    by = {}
    for prof in profs:
        by[prof] = {}
        for var in CPU_VARIANTS:
            by[prof][var] = {}
            for cs in cells:
                cell = _cpu_run(prof, var, secs, cs)
                by[prof][var][str(len(cs))] = cell
                print(f"cpu_baseline {prof} {var} {len(cs)} cores: {cell}", file=sys.stderr,
                      flush=True)
            # the reference's call form: through dispatch_func_t, one core
            cell = _cpu_run(prof, var + "_fnptr", secs, phys[:1])
            by[prof][var + "_fnptr"] = {"1": cell}
            print(f"cpu_baseline {prof} {var}_fnptr 1 core: {cell}", file=sys.stderr, flush=True)
    # every core the quota lets the job keep busy: the headline cell only
    all_cpus = (phys + [c for c in allowed if c not in set(phys)])[:quota]
    if quota > share_n:
        cell = _cpu_run(args.profile, "bit_serial", secs, all_cpus)
        by[args.profile]["bit_serial"][str(quota)] = cell
        print(f"cpu_baseline {args.profile} bit_serial {quota} cores: {cell}", file=sys.stderr,
              flush=True)
        all_note = (f"{quota} pinned processes, the job's CPU quota ({qsrc}); physical cores "
                    "first, then SMT siblings")
    else:
        all_note = (f"the job's CPU quota is {quota} CPUs ({qsrc}): every core it may keep "
                    f"busy is the {share_n}-core cell itself")
    all_cell = by[args.profile]["bit_serial"][str(max(quota, share_n))]
    share_cell = by[args.profile]["bit_serial"][str(share_n)]
    if all_cell["mpps"] < share_cell["mpps"]:
        all_note += (f"; below the {share_n}-core cell: the extra processes share cores "
                     "(SMT siblings or an over-committed quota)")
    flagged = [f"{p}/{v}/{k}" for p, vs in by.items() for v, ks in vs.items()
               for k, cell in ks.items() if "flag" in cell]
    cpu = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    head = args.profile
    one = by[head]["bit_serial_fnptr"]["1"]
    inl = by[head]["bit_serial"]["1"]
    return {
        "value": one["mpps"], "unit": "Mpkt/s", "cores": 1, "kind": "port",
        "min": one["min"], "max": one["max"], "runs": one["runs"],
        "call": "through the registered dispatcher's function pointer (process_packets, "
                "ff_dpdk_if.c:1078-1079)",
        "value_inlined": inl["mpps"],
        "sample": f"2^{CPU_SAMPLE_PKTS.bit_length() - 1} packets of each stream (4 MiB of "
                  "windows, LLC-resident as DDIO leaves an rx burst) re-run over common "
                  f"windows of ~{secs:.2f}s "
                  f"(CLOCK_MONOTONIC start and end shared by every process of a cell), median "
                  f"of {CPU_RUNS} windows per cell, one toeplitz_dispatch call per packet "
                  "(oracle restatement, gcc -O2 fs/lib flags), processes pinned one per "
                  f"physical core; host CPU: {cpu}; {len(allowed)} CPUs in the affinity "
                  f"mask, quota {quota} ({qsrc})",
        "per_gpu_share": {"value": share_cell["mpps"], "min": share_cell["min"],
                          "max": share_cell["max"], "overlap": share_cell["overlap"],
                          "unit": "Mpkt/s", "cores": share_n,
                          "note": "the 16 host cores one GPU of the box is given"},
        "all_cores": {"value": all_cell["mpps"], "min": all_cell["min"], "max": all_cell["max"],
                      "overlap": all_cell["overlap"],
                      "unit": "Mpkt/s", "cores": max(quota, share_n), "note": all_note},
        "overlap_min": OVERLAP_MIN,
        "flagged_cells": flagged,
        "by_profile": by,
    }


def probe_traffic(batches, n, stride, steps, mode=0):
    """Average duration of the ideal-traffic twin (tools/yrss_probe.hip) over
    the same buffers, rotated like the timed steps: the practical floor of the
    parse kernel on this box (mode 0).  Mode 1 moves only its reads (66 B/pkt):
    the box's streaming-read rate for the same shape."""
    import ctypes

    import torch

    lib_path = ROOT / "tools" / "libyrss_probe.so"
    if stride != 64 or not lib_path.exists():
        return None
    lib = ctypes.CDLL(str(lib_path))
    fn = lib.yrss_probe_traffic_launch_mode
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
    stream = torch.cuda.current_stream()
    args = [(w.data_ptr(), ln.data_ptr(), o.q.data_ptr(), o.hash.data_ptr(), n,
             stream.cuda_stream, mode) for w, ln, o in batches]
    for i in range(3):
        fn(*args[i % len(args)])
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(stream)
    for i in range(steps):
        fn(*args[i % len(args)])
    ev[1].record(stream)
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / steps / 1e3


def _cpulist(text: str):
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def _siblings(cpu: int):
    try:
        return _cpulist(Path(f"/sys/devices/system/cpu/cpu{cpu}/topology/"
                             "thread_siblings_list").read_text())
    except (OSError, ValueError):
        return [cpu]


def gpu_placement(device: str):
    """NUMA node of the GPU (PCI address from device_identity) and the CPU the
    host-resident dispatcher thread is pinned to: a physical core of that node
    (the first SMT sibling of its core), from the middle of the node's cores,
    never the node's first core nor that core's SMT twin (CPU 0 takes the box's
    housekeeping: the windows form's copy ran at 1256-1440 cycles a burst
    there, profiles/r04_final_bench.log; round 4's "middle of the node's CPU
    list" landed on CPU 128 / 192, the SMT twins of the nodes' first cores,
    VERDICT r04 weak 5).  The reference's dispatching lcore sits beside its
    NIC and GPU.  None where sysfs does not say."""
    node, cpu = None, None
    try:
        node = int(Path(f"/sys/bus/pci/devices/{device}.0/numa_node").read_text())
    except (OSError, ValueError):
        node = None
    allowed = sorted(os.sched_getaffinity(0))
    if node is not None and node >= 0:
        try:
            local = _cpulist(Path(f"/sys/devices/system/node/node{node}/cpulist").read_text())
            mine = [c for c in local if c in set(allowed)]
            first = set(_siblings(local[0])) if local else set()
            cores = [c for c in physical_cores(mine) if c not in first]
            cpu = cores[len(cores) // 2] if cores else (mine[len(mine) // 2] if mine else None)
        except (OSError, ValueError):
            cpu = None
    sib = _siblings(cpu) if cpu is not None else []
    return {"gpu_node": node, "dispatch_cpu": cpu, "dispatch_cpu_siblings": sib,
            "dispatch_cpu_is_first_sibling": bool(sib) and cpu == min(sib)}


def _cbench_rows(lines, keys):
    """One row per (api, burst) from YRSS_CBENCH_REPEAT runs: the median run's
    fields, its spread, and every run's rate, host cycles and placement."""
    groups = {}
    for d in lines:
        groups.setdefault((d["api"], d["burst"]), []).append(d)
    rows = []
    for (_, _), runs in groups.items():
        runs_sorted = sorted(runs, key=lambda d: d["mpps"])
        med = runs_sorted[len(runs_sorted) // 2]
        row = {k: med.get(k) for k in keys if k in med}
        row["mpps"] = med["mpps"]
        row["mpps_min"] = runs_sorted[0]["mpps"]
        row["mpps_max"] = runs_sorted[-1]["mpps"]
        row["runs"] = [{k: d.get(k) for k in ("mpps", "poll_cycles", "submit_cycles",
                                                "cpu_start", "cpu", "cpu_node", "pool_node")
                        if k in d} for d in runs]
        rows.append(row)
    return rows


def pcie_inclusive(profile: str, place=None):
    """Host-resident rates from tools/yrss_cbench (C host over the C ABI):
    DPDK-layout mbuf pool of 2^20 packets in host memory; bursts of 1024 (BASELINE's
    logical burst) and 32K with two in flight, and 1M; the persistent worker at
    F-Stack's 32-packet bursts and at 1024."""
    import subprocess

    exe = ROOT / "tools" / "yrss_cbench"
    if not exe.exists():
        return None
    place = place or {}
    pin = {} if place.get("dispatch_cpu") is None else {"YRSS_CBENCH_CPU": str(place["dispatch_cpu"])}
    out = []
    # (burst, bursts in flight over that many contexts with YRSS_F_ASYNC)
    for burst, inflight in ((1024, 2), (32768, 2), (1 << 20, 1)):
        try:
            r = subprocess.run([str(exe), str(PROFILES[profile]), str(1 << 20), str(burst), "1"],
                               capture_output=True, text=True, timeout=240,
                               env={**os.environ, **pin, "YRSS_CBENCH_MODES": "013",
                                    "YRSS_CBENCH_INFLIGHT": str(inflight)})
        except subprocess.TimeoutExpired:
            return None
        for line in r.stdout.splitlines():
            try:
                d = json.loads(line)
            except ValueError:
                continue
            out.append({"api": d["api"], "burst": d["burst"], "inflight": d.get("inflight", 1),
                        "mpps": d["mpps"], "note": d.get("note", "")})
    # persistent worker, mbuf pointers, (data, data_len) pairs and windows the
    # dispatcher copies into a registered ring ("2"), one output set per ring
    # slot: 32-packet bursts on 128 workgroups, 1024-packet bursts on 32 (the
    # best counts of the sweeps), ring depth 4 x workgroups.
    # Three runs each (median, spread), every run with its host cycles per
    # burst and the thread's and pool's NUMA placement beside the GPU's.
    # Pools: 2^20 mbufs (2.4 GB, cache-cold: every header and window a DRAM
    # miss), and 16384 mbufs, whose touched lines (4 MB) stay LLC-resident as
    # an rx ring's recycled mbufs do after rte_eth_rx_burst.  The windows
    # form's staging copy is non-temporal at 1024-packet bursts (+14 % on the
    # cold pool, no read-for-ownership of lines the GPU read), plain at 32
    # (profiles/r05_windows_copy_ab.log).
    rows = (("0", 32, 128, 1 << 20, 0), ("0", 1024, 32, 1 << 20, 0),
            ("1", 32, 128, 1 << 20, 0), ("1", 1024, 32, 1 << 20, 0),
            ("2", 32, 128, 1 << 20, 0), ("2", 1024, 32, 1 << 20, 1),
            ("1", 32, 128, 16384, 0), ("2", 32, 128, 16384, 0))
    for frames, burst, blocks, pool, win_nt in rows:
        print(f"pcie_inclusive: worker form {frames}, burst {burst}, pool {pool}", file=sys.stderr,
              flush=True)
        try:
            r = subprocess.run([str(exe), str(PROFILES[profile]), str(pool), str(burst), "1"],
                               capture_output=True, text=True, timeout=240,
                               env={**os.environ, **pin, "YRSS_CBENCH_MODES": "4",
                                    "YRSS_CBENCH_REPEAT": "3",
                                    "YRSS_CBENCH_WORKER_DEPTH": str(4 * blocks),
                                    "YRSS_CBENCH_WORKER_BLOCKS": str(blocks),
                                    "YRSS_CBENCH_WORKER_SLOTOUT": "1",
                                    "YRSS_CBENCH_WORKER_FRAMES": frames,
                                    "YRSS_CBENCH_WIN_NT": str(win_nt)})
        except subprocess.TimeoutExpired:
            break
        lines = []
        for line in r.stdout.splitlines():
            try:
                lines.append(json.loads(line))
            except ValueError:
                continue
        # bytes crossing PCIe per packet, GPU reads: mbuf pointer 8 +
        # header 64 + window 64 (64-byte packets), or pointer 8 + len 2 +
        # window 64, or len 2 + window 64; writes q 2 + hash 4 + qidx 4
        rd = {"0": 136, "1": 74, "2": 66}[frames]
        for row in _cbench_rows(lines, ("api", "burst", "inflight", "blocks", "note")):
            gbs = row["mpps"] * 1e6 * (rd + 10) / 1e9
            row.update({"pool_mbufs": pool, "pool": "cold" if pool > (1 << 16) else "llc",
                        "staging_nt": bool(win_nt) if frames == "2" else None,
                        "link_bytes_per_pkt": rd + 10, "link_GBps": round(gbs, 2),
                        "link_frac": round(gbs / PCIE_GEN5_X16_GBS, 4),
                        "gpu_node": place.get("gpu_node"),
                        "dispatch_cpu": place.get("dispatch_cpu"),
                        "dispatch_cpu_siblings": place.get("dispatch_cpu_siblings"),
                        "dispatch_cpu_is_first_sibling":
                            place.get("dispatch_cpu_is_first_sibling")})
            out.append(row)
    return out or None


def pcie_fanout(profile: str, world: int, place=None):
    """Host-resident rate of ONE dispatcher thread fanning its bursts out over
    all `world` GPUs (yrss_fanout_*, tools/yrss_cbench mode 5): the reference's
    single dispatching lcore (ff_dpdk_if.c:1653) with N PCIe links behind it.
    Run by rank 0 once every rank's device work is done."""
    import subprocess

    exe = ROOT / "tools" / "yrss_cbench"
    if not exe.exists():
        return None
    place = place or {}
    pin = {} if place.get("dispatch_cpu") is None else {"YRSS_CBENCH_CPU": str(place["dispatch_cpu"])}
    out = []
    one = bool(os.environ.get("YRSS_BENCH_ONE_DEVICE"))   # rehearsal: N contexts, device 0
    devs = ",".join("0" if one else str(d) for d in range(world))
    if one and world > 1:
        # HIP maps a process's streams on one device onto GPU_MAX_HW_QUEUES
        # (4) in-order hardware queues: N contexts' persistent workers on one
        # device would queue behind each other there.  On N devices each
        # context's streams have their own queues; the rehearsal gets one a
        # stream (two a context: its stream and its worker's).
        pin = {**pin, "GPU_MAX_HW_QUEUES": str(min(32, 2 * world + 4))}
    for frames, burst, blocks in (("1", 32, 128), ("1", 1024, 32), ("0", 32, 128)):
        if one and world > 1:
            # the N contexts' persistent workers share one GPU in the rehearsal:
            # at most 192 of its 256 CUs in all (one 1024-thread workgroup a
            # CU), so every context's workers are resident together
            blocks = max(4, min(blocks, 192 // world))
        print(f"pcie_fanout: form {frames}, burst {burst}, {blocks} workgroups a context",
              file=sys.stderr, flush=True)
        try:
            r = subprocess.run([str(exe), str(PROFILES[profile]), str(1 << 20), str(burst), "1"],
                               capture_output=True, text=True, timeout=240,
                               env={**os.environ, **pin, "YRSS_CBENCH_MODES": "5",
                                    "YRSS_CBENCH_REPEAT": "3",
                                    "YRSS_CBENCH_FANOUT_DEVICES": devs,
                                    "YRSS_CBENCH_WORKER_DEPTH": str(4 * blocks),
                                    "YRSS_CBENCH_WORKER_BLOCKS": str(blocks),
                                    "YRSS_CBENCH_WORKER_FRAMES": frames})
        except subprocess.TimeoutExpired:
            break
        lines = []
        for line in r.stdout.splitlines():
            try:
                lines.append(json.loads(line))
            except ValueError:
                continue
        for row in _cbench_rows(lines, ("api", "burst", "gpus", "inflight", "blocks")):
            # every run re-classifies the packets it covered on one context
            # (yrss_dispatch_frames) and compares q and hash packet by packet
            runs = [d for d in lines if d["api"] == row["api"] and d["burst"] == row["burst"]]
            row["checked_pkts"] = sum(d.get("checked", 0) for d in runs)
            row["mismatches"] = sum(d.get("mismatches", 0) for d in runs)
            row["gpu_node"] = place.get("gpu_node")
            row["dispatch_cpu"] = place.get("dispatch_cpu")
            row["dispatch_cpu_is_first_sibling"] = place.get("dispatch_cpu_is_first_sibling")
            out.append(row)
    return out or None


def crossover_tcp_share(cpu, pcie):
    """The hashed-TCP share of the traffic above which a host-resident GPU
    form beats ONE reference dispatcher core end to end.  The CPU's time a
    packet depends on the share s (the reference hashes TCP only,
    ff_dpdk_if.c:1986-2058): 1 / R_cpu(s) = s / R_tcp + (1 - s) / R_udp, both
    from cpu_baseline (bit-serial, through the dispatcher's function pointer,
    1 core); the GPU's rate does not depend on s (it reads every window).  So
    s* = (1 / R_gpu - 1 / R_udp) / (1 / R_tcp - 1 / R_udp), per worker row of
    pcie_inclusive (median rate): 0 when the GPU form is faster even on all-UDP
    traffic, null when it is slower even on all-TCP traffic."""
    if not cpu or not pcie:
        return None
    try:
        bp = cpu["by_profile"]
        r_udp = float(bp["udp4"]["bit_serial_fnptr"]["1"]["mpps"])
        r_tcp = float(bp["tcp4"]["bit_serial_fnptr"]["1"]["mpps"])
    except (KeyError, TypeError, ValueError):
        return None
    rows = []
    for row in pcie:
        api = row.get("api", "")
        if not api.startswith("yrss_worker") or not row.get("mpps"):
            continue
        r_gpu = float(row["mpps"])
        s = (1.0 / r_gpu - 1.0 / r_udp) / (1.0 / r_tcp - 1.0 / r_udp)
        rows.append({"api": api, "burst": row.get("burst"), "pool": row.get("pool"),
                     "gpu_mpps": r_gpu,
                     "tcp_share": None if s > 1.0 else round(max(s, 0.0), 4)})
    return {"cpu_udp_mpps": r_udp, "cpu_tcp_mpps": r_tcp, "cores": 1,
            "cpu_call": "bit-serial through the dispatcher's function pointer", "rows": rows}


def load_traffic(path: str, key: dict, field: str = "hbm_bytes_per_launch"):
    """Per-launch HBM bytes (parse kernel, or `step_hbm_bytes` for the whole
    step) from a committed PMC summary of the same workload
    (profiles/pmc_parse_hash.json), else None."""
    try:
        d = json.loads(Path(path).read_text())
    except (OSError, ValueError):
        return None
    for ent in d.get("entries", []):
        if all(ent.get("key", {}).get(k) == v for k, v in key.items()):
            return ent.get(field)
    return None


def min_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


def reduce_check(mine, world: int):
    """Every rank checks its own shard after timing; the printed line is the
    AND over ranks (one failing shard makes bit_exact false) with each rank's
    own result beside it."""
    if mine is None:
        return None
    ok = min_over_ranks(1.0 if mine["bit_exact"] else 0.0, world) > 0.5
    ranks = gather_objects(mine, world)
    return {"pkts_checked": sum(r["pkts_checked"] for r in ranks), "bit_exact": ok,
            "ranks_checked": len(ranks), "per_rank": ranks if world > 1 else None}


def check_devices(ident: str, world: int):
    """Every rank's device; N ranks must drive N distinct GPUs (except the
    declared one-device rehearsal, YRSS_BENCH_ONE_DEVICE)."""
    devs = gather_objects(ident, world)
    if len(set(devs)) != len(devs) and not os.environ.get("YRSS_BENCH_ONE_DEVICE"):
        raise SystemExit(f"bench.py: ranks share a device: {devs}")
    return devs


def dry_run(args, world, rank, local):
    """The timed loop's plumbing with the GPU work left out (--dry): spawn,
    barriers, max-over-ranks time, sum of packets, device check.  For CPU
    tests of the N>1 launch; the line says dry and carries no value."""
    devices = check_devices(device_identity(local, True), world)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    t1 = time.perf_counter()
    barrier(world)
    elapsed = max_over_ranks(t1 - t0, world)
    total = sum_over_ranks(float(args.pkts * args.steps), world)
    # the check's plumbing: each rank compares its shard's oracle answer with
    # itself (no device), YRSS_BENCH_DRY_FAIL_RANK marks one rank's shard bad
    mine = None
    if args.check:
        mine = {"rank": rank, "device": devices[rank], "pkts_checked": min(args.check, args.pkts),
                "bit_exact": os.environ.get("YRSS_BENCH_DRY_FAIL_RANK") != str(rank)}
    check = reduce_check(mine, world)
    cpu = cpu_baseline(args, args.nb_queues or args.nb_procs) \
        if rank == 0 and args.cpu_seconds > 0 else None
    barrier(world)
    if rank == 0:
        print(json.dumps({"metric": "dry run (no GPU work)", "dry": True, "value": None,
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "pkts_total": total, "elapsed_s": elapsed,
                          "config": {"parallelism": f"shard{world}", "devices": devices},
                          "cpu_baseline": cpu, "check": check}),
              flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


EXTRA_LABELS = {"vlan6_tcp": "configs[3]", "jumbo_tcp4": "configs[4]", "imix": "configs[2]",
                "udp4": "configs[1]"}


def run_extra_config(eng, profile, args, world, rank, devices):
    """One more BASELINE config after the headline: each rank classifies its own
    --pkts shard of `profile` (weak scaling, no collective on the data path),
    timed like the headline (barrier + synchronize on both sides, max over
    ranks) over min(steps, 50) steps of four rotated batches after min(warmup,
    20) untimed ones, as the headline rotates its batches; the parse kernel
    timed by events on its own dispatch packet; then checked against the oracle
    (q and hash of the first --check packets, the whole per-queue lists)."""
    import numpy as np
    import torch

    from oracle import oracle
    from yastack_amd import abi

    n = args.pkts
    nbq = args.nb_queues or args.nb_procs
    nbat = 4
    bats = []
    for k in range(nbat):
        w_k, l_k = eng.synth(PROFILES[profile], n, (rank * nbat + k) * n, SEED, NFLOWS[profile],
                             args.stride)
        bats.append((w_k, l_k, eng.alloc_out(n, w_k.device)))
    it = [0]

    def step():
        w_k, l_k, o_k = bats[it[0] % nbat]
        it[0] += 1
        eng.dispatch_dev(w_k, l_k, args.stride, n, out=o_k)

    for _ in range(max(5, min(args.warmup, 20))):
        step()
    torch.cuda.synchronize()
    steps = max(1, min(args.steps, 50))
    eng.timing_enable(1 << abi.K_PARSE_HASH)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    elapsed = max_over_ranks(t1 - t0, world)
    k_ms, k_cnt = eng.timing_read(abi.K_PARSE_HASH)
    eng.timing_enable(0)
    k_s = max_over_ranks(k_ms / max(k_cnt, 1) / 1e3, world)
    # the check, on the batch the last step classified
    w_k, l_k, o_k = bats[(it[0] - 1) % nbat]
    m = min(args.check or (1 << 20), n)
    c = oracle.cfg(args.nb_procs, nbq, 1, args.dispatch_only_core)
    q_ref, h_ref = oracle.dispatch_windows(w_k[: m * args.stride].cpu().numpy(), args.stride,
                                           l_k[:m].cpu().numpy().view(np.uint16), c)
    ok = bool(np.array_equal(o_k.q[:m].cpu().numpy(), q_ref) and
              np.array_equal(o_k.hash[:m].cpu().numpy().view(np.uint32), h_ref))
    qi_ref, qs_ref = oracle.process_burst(o_k.q[:n].cpu().numpy(), nbq)
    ok = ok and bool(np.array_equal(o_k.qstart.cpu().numpy().view(np.uint32), qs_ref) and
                     np.array_equal(o_k.qidx[:n].cpu().numpy().view(np.uint32), qi_ref))
    chk = reduce_check({"rank": rank, "device": devices[rank], "pkts_checked": m,
                        "bit_exact": ok}, world)
    del bats
    total = sum_over_ranks(float(n * steps), world)
    bpp = min(args.stride, 64) + 2 + 4 + 2
    return {"config": EXTRA_LABELS.get(profile, profile), "profile": profile,
            "workload": WORKLOADS[profile], "nflows": NFLOWS[profile], "n_gpus": world,
            "pkts_per_gpu": n, "steps": steps,
            "value": round(total / elapsed / 1e6, 2), "unit": "Mpkt/s",
            "ms_per_step": round(elapsed / steps * 1e3, 4),
            "parse_us": round(k_s * 1e6, 2),
            "outside_parse_us": round(elapsed / steps * 1e6 - k_s * 1e6, 2) if k_s else None,
            "roofline_frac": round(bpp * n / k_s / 1e9 / HBM_PEAK_GBS, 4) if k_s else None,
            "ranks_checked": chk["ranks_checked"], "bit_exact": chk["bit_exact"],
            "pkts_checked": chk["pkts_checked"]}


def main(argv=None):
    raw = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(raw)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus, raw)
    world, rank, local = dist_setup(args.gpus)
    if args.dry:
        return dry_run(args, world, rank, local)
    import numpy as np
    import torch

    from yastack_amd import SoftRss, abi
    from yastack_amd.shard import shard_range

    # a launcher that gives each rank only its own GPU (HIP_VISIBLE_DEVICES per
    # rank) leaves that GPU at ordinal 0; device_count() does not open the device
    nvis = torch.cuda.device_count()
    if nvis == 0:
        raise SystemExit("bench.py: no GPU visible")
    if local >= nvis:
        local = local % nvis
    torch.cuda.set_device(local)
    devices = check_devices(device_identity(local, False), world)
    nbq = args.nb_queues or args.nb_procs
    hooks = {k: int(v) for k, v in (kv.split("=") for kv in args.test_hooks.split(",") if kv)}
    eng = SoftRss(nb_procs=args.nb_procs, nb_queues=nbq, soft_dispatch=1,
                  dispatch_only_core=args.dispatch_only_core, device=local, max_burst=0,
                  lib_path=str(abi.TEST_LIB_PATH) if hooks else None)
    if "merge" in hooks:
        abi.check(eng._lib.yrss_debug_partial_merge(eng._ctx, hooks["merge"]), "partial_merge")
    if "groups" in hooks:
        abi.check(eng._lib.yrss_debug_line_groups(eng._ctx, hooks["groups"], 0), "line_groups")
    if args.tune:
        eng.set_tuning(**{k: int(v) for k, v in (kv.split("=") for kv in args.tune.split(","))})
    n = args.pkts
    nbat = max(1, args.batches)
    prof = PROFILES[args.profile]
    # weak scaling: rank r owns shards [r*nbat, (r+1)*nbat) of one packet stream;
    # step i classifies batch i mod nbat, so no step re-reads what the previous
    # nbat-1 steps left in the caches
    batches = []
    for k in range(nbat):
        w_k, l_k = eng.synth(prof, n, (rank * nbat + k) * n, SEED, NFLOWS[args.profile],
                             args.stride)
        o_k = eng.alloc_out(n, w_k.device, want_hash=True, compact=not args.no_compact,
                            want_filter=args.filter)
        batches.append((w_k, l_k, o_k))
    win, lens, out = batches[0]
    if args.filter:
        eng.set_kni(True, "reject", "80,443,8000-8080", "53,123")
    torch.cuda.synchronize()
    it = [0]

    def step():
        w_k, l_k, o_k = batches[it[0] % nbat]
        it[0] += 1
        eng.dispatch_dev(w_k, l_k, args.stride, n, out=o_k, compact=not args.no_compact)

    probe_s = probe_traffic(batches, n, args.stride, max(args.steps, 10))
    probe_rd_s = probe_traffic(batches, n, args.stride, max(args.steps, 10), mode=1)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # events ride on the dominant kernel's dispatch packet (hipExtLaunchKernel)
    eng.timing_enable((1 << abi.K_PARSE_HASH) if args.kernel_timing else 0)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    elapsed = max_over_ranks(t1 - t0, world)
    k_ms, k_cnt = eng.timing_read(abi.K_PARSE_HASH)
    k_avg_s = max_over_ranks(k_ms / max(k_cnt, 1) / 1e3, world)
    k_med_s = max_over_ranks(eng.timing_quantile(abi.K_PARSE_HASH) / 1e3, world) \
        if k_cnt else 0.0
    eng.timing_enable(0)
    # the scan and scatter shares, from a separate pass after the timed one:
    # events on all three kernels widen the step by ~9 us, so the timed steps
    # carry them on the parse kernel only
    side_us = {}
    if not args.no_compact and args.kernel_timing:
        eng.timing_enable((1 << abi.K_SCAN) | (1 << abi.K_SCATTER))
        for _ in range(min(args.steps, 20)):
            step()
        torch.cuda.synchronize()
        for name, k in (("scan", abi.K_SCAN), ("scatter", abi.K_SCATTER)):
            ms, cnt = eng.timing_read(k)
            side_us[name] = round(max_over_ranks(ms / max(cnt, 1) / 1e3, world) * 1e6, 2)
        eng.timing_enable(0)

    total_pkts = sum_over_ranks(float(n * args.steps), world)
    value = total_pkts / elapsed / 1e6
    # algorithmic bytes per packet for the parse kernel: header window read
    # (min(stride, 64) — the kernel stages 64 B), data_len read (2), hash (4) and
    # queue (2) written = 72 B at 64-B windows.
    bpp = min(args.stride, 64) + 2 + 4 + 2 + (1 if args.filter else 0)
    achieved = bpp * n / k_avg_s / 1e9 if k_avg_s > 0 else 0.0
    # the whole step: the same bytes plus the per-queue index lists (4 B/pkt
    # written, SURVEY §8(d): "report B=76 in that mode") over ms_per_step
    step_s = elapsed / args.steps
    step_bpp = bpp + (0 if args.no_compact else 4)
    step = {"bytes_per_pkt": step_bpp, "achieved": round(step_bpp * n / step_s / 1e9, 1),
            "frac": round(step_bpp * n / step_s / 1e9 / HBM_PEAK_GBS, 4),
            "parse_us": round(k_avg_s * 1e6, 2), **{f"{k}_us": v for k, v in side_us.items()},
            "outside_parse_us": round((step_s - k_avg_s) * 1e6, 2)}
    key = {"profile": args.profile, "pkts": n, "stride": args.stride,
           "compact": not args.no_compact}
    traffic = load_traffic(args.pmc, key)
    step["traffic"] = load_traffic(args.pmc, key, "step_hbm_bytes")

    check = None
    if args.check:
        from oracle import oracle

        m = min(args.check, n)
        c = oracle.cfg(args.nb_procs, nbq, 1, args.dispatch_only_core)
        w_h = win[: m * args.stride].cpu().numpy()
        l_h = lens[:m].cpu().numpy().view(np.uint16)
        q_ref, h_ref = oracle.dispatch_windows(w_h, args.stride, l_h, c)
        ok = bool(np.array_equal(out.q[:m].cpu().numpy(), q_ref) and
                  np.array_equal(out.hash[:m].cpu().numpy().view(np.uint32), h_ref))
        if not args.no_compact:
            q_all = out.q[:n].cpu().numpy()
            qi_ref, qs_ref = oracle.process_burst(q_all, nbq)
            ok = ok and bool(np.array_equal(out.qstart.cpu().numpy().view(np.uint32), qs_ref) and
                             np.array_equal(out.qidx[:n].cpu().numpy().view(np.uint32), qi_ref))
        check = {"rank": rank, "device": devices[rank], "pkts_checked": m, "bit_exact": ok,
                 "parse_us": round(k_ms / max(k_cnt, 1) * 1e3, 2)}
    check = reduce_check(check, world)

    # the 8-GPU configs (and any other asked for), each rank its own shard,
    # after the headline: a line for configs[3] / configs[4] at every N
    extra = None
    if args.extra_configs and not args.no_compact and not args.filter:
        del batches, win, lens, out
        torch.cuda.empty_cache()
        extra = []
        for p in [x for x in args.extra_configs.split(",") if x]:
            extra.append(run_extra_config(eng, p, args, world, rank, devices))
            if rank == 0:
                print(f"configs_extra: {extra[-1]}", file=sys.stderr, flush=True)

    # the CPU baseline on rank 0 once every rank's device work is done (at any
    # N: the other ranks wait at the barrier)
    barrier(world)
    cpu = None
    if rank == 0 and args.cpu_seconds > 0:
        cpu = cpu_baseline(args, nbq)
    barrier(world)
    pcie = fan = None
    if args.pcie:
        barrier(world)                    # every rank's device work is done
        if rank == 0:
            eng.close()                   # release the device buffers first
            place = gpu_placement(devices[0])
            if world == 1:
                pcie = pcie_inclusive(args.profile, place)
            fan = pcie_fanout(args.profile, world, place)
        barrier(world)

    if rank == 0:
        line = {
            "metric": "Mpkt/s device-resident soft-RSS parse+hash, 64B pkts, 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "Mpkt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (on-device counter-based generator, include/yrss_synth.h)",
            "config": {
                "workload": WORKLOADS[args.profile],
                "pkts_per_gpu": n, "logical_burst": 1024, "win_stride": args.stride,
                "distinct_batches": nbat,
                "nb_procs": args.nb_procs, "nb_queues": nbq, "soft_dispatch": 1,
                "dispatch_only_core": args.dispatch_only_core,
                "per_queue_lists": not args.no_compact,
                "kni_filter": args.filter,
                "test_hooks": hooks or None,
                "parallelism": f"shard{world}",
                "devices": devices,
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "yrss_parse_hash", "bytes_per_pkt": bpp,
                "kernel_avg_us": round(k_avg_s * 1e6, 2),
                "kernel_median_us": round(k_med_s * 1e6, 2),
                "step": step,
                "probe": None if probe_s is None else {
                    "what": "ideal-traffic twin (tools/yrss_probe.hip): same bytes, no parse",
                    "us": round(probe_s * 1e6, 2),
                    "achieved": round(bpp * n / probe_s / 1e9, 1),
                    "parse_frac_of_probe": round(probe_s / k_avg_s, 4) if k_avg_s else None,
                    "reads_only_us": round(probe_rd_s * 1e6, 2) if probe_rd_s else None,
                    "reads_only_achieved": round((bpp - 6) * n / probe_rd_s / 1e9, 1)
                    if probe_rd_s and not args.filter else None},
            },
            "configs_extra": extra,
            "cpu_baseline": cpu,
            "pcie_inclusive": pcie,
            "pcie_inclusive_crossover_tcp_share": crossover_tcp_share(cpu, pcie),
            "pcie_fanout": fan,
            "check": check,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    if len(sys.argv) == 3 and sys.argv[1] == "--cpu-worker":
        sys.exit(cpu_worker(sys.argv[2]))
    sys.exit(main() or 0)
