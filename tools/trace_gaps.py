#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: per-kernel mean duration and the mean
idle gap before each kernel (end of the previous dispatch on the same queue to
the start of this one).

    python tools/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv [--skip 5]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=5, help="leading dispatches per kernel to drop")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    dur, gap, seen = defaultdict(list), defaultdict(list), defaultdict(int)
    prev_end = {}
    for r in rows:
        name = r["Kernel_Name"].replace("void ", "").replace(
            "(anonymous namespace)::", "").split("(")[0].split("<")[0]
        q = r.get("Queue_Id", "0")
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        seen[name] += 1
        if seen[name] > a.skip:
            dur[name].append((e - s) / 1e3)
            if q in prev_end and 0 <= s - prev_end[q] < 50_000:
                gap[name].append((s - prev_end[q]) / 1e3)
        prev_end[q] = e
    print(f"{'kernel':40s} {'n':>5s} {'mean_us':>9s} {'gap_before_us':>14s}")
    for k in dur:
        g = sum(gap[k]) / len(gap[k]) if gap[k] else float("nan")
        print(f"{k[:40]:40s} {len(dur[k]):5d} {sum(dur[k]) / len(dur[k]):9.2f} {g:14.2f}")


if __name__ == "__main__":
    main()
