"""bench.py's N-rank launch on CPU (--dry: no GPU work).

`python bench.py --gpus N` with no launcher must start N ranks itself (the
driver's 1/2/4/8 curve would otherwise measure one GPU), every rank must
report its own device, and a --gpus / WORLD_SIZE mismatch must fail.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
DIST_VARS = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT",
             "YRSS_BENCH_ONE_DEVICE")


def _run(args, extra_env=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in DIST_VARS}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=timeout)


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_gpus2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--dry", "--steps", "3", "--warmup", "0", "--pkts", "1000",
              "--cpu-seconds", "0"])
    assert r.returncode == 0, r.stderr
    d = _line(r.stdout)
    assert d["dry"] is True and d["value"] is None
    assert d["n_gpus"] == 2
    devs = d["config"]["devices"]
    assert len(devs) == 2 and len(set(devs)) == 2
    assert d["pkts_total"] == 2 * 3 * 1000


def test_gpus1_single_rank():
    r = _run(["--gpus", "1", "--dry", "--steps", "2", "--warmup", "0", "--cpu-seconds", "0"])
    assert r.returncode == 0, r.stderr
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and len(d["config"]["devices"]) == 1


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--dry"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


def test_shared_device_refused():
    # two ranks claiming one device (no rehearsal flag) must not produce a line
    r = _run(["--gpus", "2", "--dry", "--steps", "1", "--cpu-seconds", "0"], {"YRSS_BENCH_FAKE_SAME_DEVICE": "1"})
    assert r.returncode != 0
    assert "share a device" in r.stderr


def test_torchrun_two_ranks():
    """The driver's form for N > 1: torch.distributed.run sets WORLD_SIZE /
    RANK / LOCAL_RANK and bench.py runs as one of its ranks."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in DIST_VARS}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(port), str(ROOT / "bench.py"), "--gpus", "2",
                        "--dry", "--steps", "2", "--warmup", "0", "--pkts", "500",
                        "--cpu-seconds", "0"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and len(set(d["config"]["devices"])) == 2
    assert d["pkts_total"] == 2 * 2 * 500


def test_two_ranks_check_and_cpu_baseline():
    """N > 1 line: bit_exact is the AND over every rank's own shard check (a
    failing rank 1 turns it false), each rank's result is listed, and the CPU
    baseline is present at n_gpus 2 (rank 0, after the device work)."""
    base = ["--gpus", "2", "--dry", "--steps", "2", "--warmup", "0", "--pkts", "4096",
            "--check", "4096", "--cpu-seconds", "1"]
    r = _run(base, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2
    assert d["check"]["bit_exact"] is True and d["check"]["ranks_checked"] == 2
    assert d["check"]["pkts_checked"] == 2 * 4096
    assert [x["rank"] for x in d["check"]["per_rank"]] == [0, 1]
    cpu = d["cpu_baseline"]
    assert cpu and cpu["value"] > 0 and cpu["cores"] == 1 and cpu["all_cores"]["cores"] >= 1
    r = _run(base[:-2] + ["--cpu-seconds", "0"], {"YRSS_BENCH_DRY_FAIL_RANK": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["check"]["bit_exact"] is False
    assert [x["bit_exact"] for x in d["check"]["per_rank"]] == [True, False]
