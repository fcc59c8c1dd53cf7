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
    assert p == {"gpu_node": None, "dispatch_cpu": None}


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
    q, _ = bench.cpu_quota()
    assert cpu["all_cores"]["cores"] == max(q, cpu["per_gpu_share"]["cores"])
    assert "quota" in cpu["all_cores"]["note"]
    json.dumps(cpu)
