"""bench.py's host-side helpers, no GPU: the CPU quota and core choice of the
CPU baseline, every cell a median of several timed windows with its spread,
and the host-resident rows folded into median + spread + per-run placement."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_cpulist_parses_sysfs_ranges():
    assert bench._cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert bench._cpulist("5") == [5]
    assert bench._cpulist("") == []


def test_cpu_quota_is_within_the_affinity_mask():
    n, src = bench.cpu_quota()
    assert 1 <= n <= len(os.sched_getaffinity(0))
    assert isinstance(src, str) and src


def test_physical_cores_one_per_core():
    cpus = sorted(os.sched_getaffinity(0))
    phys = bench.physical_cores(cpus)
    assert phys and len(phys) <= len(cpus) and len(set(phys)) == len(phys)
    assert set(phys) <= set(cpus)


def test_cbench_rows_median_and_spread():
    runs = [{"api": "yrss_worker_submit_frames", "burst": 32, "inflight": 512, "blocks": 128,
             "mpps": v, "poll_cycles": 400 + i, "submit_cycles": 80, "cpu_start": 3, "cpu": 3,
             "cpu_node": 0, "pool_node": [0, 0], "note": "n"} for i, v in enumerate((150.0, 40.9,
                                                                                    170.0))]
    runs.append(dict(runs[0], burst=1024, mpps=260.0))
    rows = bench._cbench_rows(runs, ("api", "burst", "inflight", "blocks", "note"))
    r32 = [r for r in rows if r["burst"] == 32][0]
    assert r32["mpps"] == 150.0 and r32["mpps_min"] == 40.9 and r32["mpps_max"] == 170.0
    assert len(r32["runs"]) == 3 and r32["runs"][1]["poll_cycles"] == 401
    assert r32["runs"][0]["pool_node"] == [0, 0]
    r1k = [r for r in rows if r["burst"] == 1024][0]
    assert r1k["mpps"] == r1k["mpps_min"] == r1k["mpps_max"] == 260.0


def test_gpu_placement_unknown_device():
    p = bench.gpu_placement("ffff:ff:ff")
    assert p["gpu_node"] is None and p["dispatch_cpu"] is None


def test_gpu_placement_takes_a_physical_core_off_the_first(monkeypatch, tmp_path):
    """The dispatcher goes on a physical core of the GPU's node (the first SMT
    sibling of its core), never the node's first core nor that core's twin
    (CPU 128 / 192 were the twins of CPUs 0 / 64)."""
    sysfs = {"/sys/bus/pci/devices/0000:0d:00.0/numa_node": "0\n",
             "/sys/devices/system/node/node0/cpulist": "0-7,16-23\n"}
    for c in range(8):   # cores 0..7, twins 16..23
        for cpu in (c, c + 16):
            sysfs[f"/sys/devices/system/cpu/cpu{cpu}/topology/thread_siblings_list"] = \
                f"{c},{c + 16}\n"
    real = bench.Path

    class FakePath(type(real())):
        def read_text(self):
            key = str(self)
            if key in sysfs:
                return sysfs[key]
            raise OSError(key)

    monkeypatch.setattr(bench, "Path", FakePath)
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(32)))
    p = bench.gpu_placement("0000:0d:00")
    assert p["gpu_node"] == 0
    assert p["dispatch_cpu"] in range(1, 8) and p["dispatch_cpu_is_first_sibling"]
    assert p["dispatch_cpu_siblings"] == [p["dispatch_cpu"], p["dispatch_cpu"] + 16]


def test_cpu_worker_windows_are_common():
    """Every process of a multi-core cell runs over one CLOCK_MONOTONIC window
    (VERDICT r04 weak 6): two processes, overlap near 1, and a cell below
    OVERLAP_MIN would carry a flag."""
    cell = bench._cpu_run("udp4", "table", 0.3, ["-", "-"], runs=2)
    assert cell["runs"] == 2 and cell["overlap"] > 0.5
    assert ("flag" in cell) == (cell["overlap"] < bench.OVERLAP_MIN)


def test_cpu_baseline_cells_carry_spread():
    """Two cores, a short window: every cell is a median with min/max over
    CPU_RUNS windows; all_cores states the quota it was sized by."""
    args = bench.parse_args(["--cpu-seconds", "0.3"])
    cpu = bench.cpu_baseline(args, 3)
    assert cpu["kind"] == "port" and cpu["cores"] == 1 and cpu["runs"] == bench.CPU_RUNS
    assert cpu["min"] <= cpu["value"] <= cpu["max"]
    for prof, by_var in cpu["by_profile"].items():
        for var, cells in by_var.items():
            for cores, cell in cells.items():
                assert cell["min"] <= cell["mpps"] <= cell["max"], (prof, var, cores, cell)
                assert cell["runs"] == bench.CPU_RUNS and 0.0 <= cell["overlap"] <= 1.0
    # the reference's call form (function pointer) and the inlined one, 1 core
    head = cpu["by_profile"][args.profile]
    assert cpu["value"] == head["bit_serial_fnptr"]["1"]["mpps"]
    assert cpu["value_inlined"] == head["bit_serial"]["1"]["mpps"]
    assert isinstance(cpu["flagged_cells"], list)
    q, _ = bench.cpu_quota()
    assert cpu["all_cores"]["cores"] == max(q, cpu["per_gpu_share"]["cores"])
    assert "quota" in cpu["all_cores"]["note"]
    json.dumps(cpu)
