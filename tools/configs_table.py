#!/usr/bin/env python3
"""Run bench.py once per BASELINE.json config on one GPU and print a table.

Each row: device-resident Mpkt/s, parse-kernel HBM fraction, fraction of the
ideal-traffic probe, and the CPU baseline (oracle port, 1 core) on the same
synthetic stream.  Writes gpurun_out/configs.json.

    python tools/configs_table.py [--steps 50] [--cpu-seconds 5]
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

CONFIGS = [
    ("1", "udp4_1flow", "64B UDP/IPv4, 1 flow (CPU-only config in BASELINE)", []),
    ("2", "udp4", "64B UDP/IPv4, 1M flows, burst 1024", []),
    ("3", "imix", "IMIX 64/570/1500 7:4:1 TCP+UDP, 1M flows", []),
    ("4", "vlan6_tcp", "64B VLAN+IPv6+TCP, 4M flows", []),
    ("5", "jumbo_tcp4", "9000B jumbo TCP/IPv4 (data_len 2048), 16M flows", []),
    ("-", "tcp4", "64B TCP/IPv4, 1M flows (all hashed)", []),
]
# the same all-hashed stream over more dispatch queues (nb_procs lcores,
# dispatch_only_core): the line scatter at 8192-packet spans up to 128
# buckets (packed ranks), 16 384-packet spans beyond (yrss.hip)
QUEUES = [
    ("q8", "tcp4", "64B TCP/IPv4, nb_procs 8 (9 buckets)", ["--nb-procs", "8"]),
    ("q16", "tcp4", "64B TCP/IPv4, nb_procs 16 (17 buckets)", ["--nb-procs", "16"]),
    ("q32", "tcp4", "64B TCP/IPv4, nb_procs 32 (33 buckets)", ["--nb-procs", "32"]),
    ("q64", "tcp4", "64B TCP/IPv4, nb_procs 64 (65 buckets)", ["--nb-procs", "64"]),
    ("q255", "tcp4", "64B TCP/IPv4, nb_procs 255 (256 buckets, 16 384-packet spans, rank beside q)", ["--nb-procs", "255"]),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "configs.json"))
    ap.add_argument("--queues", type=int, default=1, help="also the nb_procs sweep (QUEUES)")
    args = ap.parse_args()
    rows = []
    for cid, prof, desc, extra in CONFIGS + (QUEUES if args.queues else []):
        cmd = [sys.executable, str(ROOT / "bench.py"), "--profile", prof, "--steps",
               str(args.steps), "--cpu-seconds", str(args.cpu_seconds if not extra else 0),
               "--pcie", "0", "--extra-configs=", *extra]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        line = next((ln for ln in r.stdout.splitlines() if ln.startswith("{")), None)
        if r.returncode != 0 or line is None:
            print(f"config {cid} failed:\n{r.stderr[-2000:]}", file=sys.stderr)
            sys.exit(1)
        d = json.loads(line)
        rf = d["roofline"]
        row = {"config": cid, "profile": prof, "desc": desc, "mpps": d["value"],
               "ms_per_step": d["ms_per_step"], "kernel_us": rf["kernel_avg_us"],
               "hbm_frac": rf["frac"],
               "probe_frac": (rf.get("probe") or {}).get("parse_frac_of_probe"),
               "cpu_mpps": (d.get("cpu_baseline") or {}).get("value"),
               "bit_exact": (d.get("check") or {}).get("bit_exact")}
        rows.append(row)
        print(json.dumps(row), flush=True)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(rows, indent=1))
    print("| cfg | workload | GPU Mpkt/s | parse kernel µs | HBM frac | probe frac | CPU Mpkt/s (1 core) | bit-exact |")
    print("|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['config']} | {r['desc']} | {r['mpps']:.0f} | {r['kernel_us']:.1f} | "
              f"{r['hbm_frac']:.3f} | {r['probe_frac']} | {r['cpu_mpps']} | {r['bit_exact']} |")


if __name__ == "__main__":
    main()
