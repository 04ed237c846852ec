#!/usr/bin/env python3
"""One summary row per bench line found in the given log files (the JSON
line bench.py prints): kernel avg, roofline fraction, value, verify."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        r = d["roofline"]
        v = d.get("verify") or {}
        print("%-28s %-8s kernel %7.2f us  frac %.3f  value %8.1f  step %8.2f us  verify %s / %s (graph)  eager %s"
              % (path.split("/")[-1], d["config"].get("config"), r["kernel_avg_us"], r["frac"], d["value"],
                 d["ms_per_step"] * 1e3, v.get("kernel_avg_us"), v.get("graph_kernel_avg_us"),
                 None if d.get("eager_ms_per_step") is None else round(d["eager_ms_per_step"] * 1e3, 2)))
