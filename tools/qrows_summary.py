#!/usr/bin/env python3
"""Summarise gpurun_out/qrows_<tag>.log files (tools/gpu_r03_qrows.sh): one
row per queue count with the step, each kernel's time and the check."""
import json
import sys

for tag in sys.argv[1:]:
    txt = open(f"gpurun_out/qrows_{tag}.log").read()
    print(f"[{tag}]")
    for blk in txt.split("== ")[1:]:
        name = blk.split("\n")[0]
        for ln in blk.splitlines():
            if ln.startswith("{"):
                d = json.loads(ln)
                s = d["roofline"]["step"]
                ck = d["check"]["bit_exact"] if d.get("check") else None
                print(f"  {name:12s} {d['value']:9.0f} Mpkt/s  step {d['ms_per_step']:.4f} ms  parse "
                      f"{s['parse_us']:6.1f}  scan {s.get('scan_us')}  scatter {s.get('scatter_us')}"
                      f"  bit_exact {ck}")
            elif ln.startswith('"') and "probe" not in ln and "synth" not in ln and "Name" not in ln:
                f = ln.split('",')
                print(f"      {f[0][1:60]:60s} avg {float(f[1].split(',')[2]) / 1e3:8.2f} us")
