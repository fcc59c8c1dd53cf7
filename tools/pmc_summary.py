#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into per-launch HBM bytes for bench.py.

Reads the counter_collection CSVs of two separate rocprofv3 runs of the same
bench command (one with --pmc FETCH_SIZE, one with --pmc WRITE_SIZE) and
writes/updates profiles/pmc_parse_hash.json:

  hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024

FETCH_SIZE/WRITE_SIZE are in KiB.  The factor 2 on FETCH_SIZE is the gfx950
correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE reads exactly half the
bytes of a wide 16-B/lane coalesced streaming read — the window loads here).
Raw values are kept next to the corrected total.

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR --profile udp4 --pkts N \
        --stride 64 [--compact 1]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def per_kernel(dirpath: str, counter: str) -> dict:
    files = glob.glob(f"{dirpath}/**/*counter_collection*.csv", recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {dirpath}")
    acc: dict[str, list[float]] = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                acc.setdefault(name, []).append(float(row["Counter_Value"]))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--profile", default="udp4")
    ap.add_argument("--pkts", type=int, default=1 << 24)
    ap.add_argument("--stride", type=int, default=64)
    ap.add_argument("--compact", type=int, default=1)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "pmc_parse_hash.json"))
    args = ap.parse_args()

    fetch = per_kernel(args.fetch_dir, "FETCH_SIZE")
    write = per_kernel(args.write_dir, "WRITE_SIZE")
    summary = {}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        summary[name] = {"dispatches": max(len(f), len(w)), "fetch_kib_raw": fk,
                         "write_kib": wk}
    parse = [k for k in summary if "yrss_parse_hash" in k]
    if not parse:
        raise SystemExit("yrss_parse_hash not found in PMC output")
    ent = summary[parse[0]]
    hbm = (2 * ent["fetch_kib_raw"] + ent["write_kib"]) * 1024
    algo = (min(args.stride, 64) + 8) * args.pkts
    entry = {
        "key": {"profile": args.profile, "pkts": args.pkts, "stride": args.stride,
                "compact": bool(args.compact)},
        "kernel": parse[0],
        "fetch_kib_raw": ent["fetch_kib_raw"], "write_kib": ent["write_kib"],
        "hbm_bytes_per_launch": round(hbm),
        "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": round(hbm / algo, 4),
        "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) KiB; x2 on FETCH per MI355X_MICROARCH §HBM",
        "all_kernels": summary,
    }
    # the whole step (SURVEY 8(d) "B=76 in that mode"): parse (corrected as
    # above) + scan + scatter, whose reads are not 16-B/lane streams, so their
    # FETCH_SIZE is taken as measured
    side = [k for k in summary if "yrss_seg_scan" in k or "yrss_scatter" in k]
    if side and args.compact:
        step = hbm + sum(((summary[k]["fetch_kib_raw"] or 0) + (summary[k]["write_kib"] or 0))
                         * 1024 for k in side)
        step_algo = (min(args.stride, 64) + 12) * args.pkts
        entry["step_hbm_bytes"] = round(step)
        entry["step_algorithmic_bytes"] = step_algo
        entry["step_traffic_over_algorithmic"] = round(step / step_algo, 4)
    out = Path(args.out)
    data = json.loads(out.read_text()) if out.exists() else {"entries": []}
    data["entries"] = [e for e in data["entries"] if e.get("key") != entry["key"]] + [entry]
    out.write_text(json.dumps(data, indent=1) + "\n")
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
