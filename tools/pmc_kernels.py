#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one or more pass
directories): counter value per dispatch, averaged over the dispatches of each
kernel, plus derived rows (HBM bytes per dispatch with the gfx950 FETCH_SIZE
x2 correction of MI355X_MICROARCH.md, wave-cycle split, LDS conflict share).

    python tools/pmc_kernels.py DIR [DIR ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    for k in ("yrss_parse_hash", "yrss_seg_scan", "yrss_scatter_lines", "yrss_scatter_wide",
              "yrss_scatter", "list_writes",
              "yrss_synth", "probe"):
        if k in name:
            return k + ("<" + name.split("<", 1)[1].split(">")[0] + ">" if "<" in name else "")
    return name[:40]


def main():
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> per-dispatch values
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    key = (row.get("Dispatch_Id"), short(row["Kernel_Name"]), row["Counter_Name"])
                    per[key] += float(row["Counter_Value"])
            for (_, k, c), v in per.items():
                vals[k][c].append(v)
    for k in sorted(vals):
        if not any(s in k for s in ("parse", "scan", "scatter", "list_writes")):
            continue
        c = {n: sum(v) / len(v) for n, v in vals[k].items()}
        print(f"  {k}")
        for n in sorted(c):
            print(f"    {n:24s} {c[n]:16.1f}")
        if "FETCH_SIZE" in c:
            print(f"    {'hbm_read_MB(x2 corr)':24s} {2 * c['FETCH_SIZE'] * 1024 / 1e6:16.2f}")
        if "WRITE_SIZE" in c:
            print(f"    {'hbm_write_MB':24s} {c['WRITE_SIZE'] * 1024 / 1e6:16.2f}")
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            w = c["SQ_WAVE_CYCLES"]
            print(f"    wave-cycle split: active {c.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f} "
                  f"parked {c.get('SQ_WAIT_ANY', 0) / w:.2f} issue-stall "
                  f"{c.get('SQ_WAIT_INST_ANY', 0) / w:.2f}")
        if "SQ_LDS_IDX_ACTIVE" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            print(f"    lds conflict share {c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:.3f}")


if __name__ == "__main__":
    main()
