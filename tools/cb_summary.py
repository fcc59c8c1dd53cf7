#!/usr/bin/env python3
"""One line per yrss_cbench JSON record: api, burst, bursts in flight, rate."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        try:
            d = json.loads(line)
        except ValueError:
            continue
        extra = ""
        if "poll_cycles" in d:   # host TSC cycles per burst inside poll / submit
            extra = "  poll %5.0f cyc  submit %5.0f cyc" % (d["poll_cycles"], d["submit_cycles"])
        print("%-26s burst %7d inflight %d %9.2f Mpkt/s %9.2f us/burst%s"
              % (d["api"], d["burst"], d.get("inflight", 1), d["mpps"], d["us_per_burst"], extra))
