#!/usr/bin/env python3
"""Summarise gpurun_out/ logs: bench JSON lines and kbench variant tables."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in sorted(glob.glob(os.path.join(d, "*.log"))):
    for line in open(f, errors="replace"):
        line = line.strip()
        if not line.startswith("{"):
            continue
        try:
            j = json.loads(line)
        except Exception:
            continue
        name = os.path.basename(f)
        if "roofline" in j:
            r = j["roofline"]
            v = j.get("verify") or {}
            print("%-22s %-8s value %8.1f GiB/s step %7.2f us kernel %7.2f us frac %.4f exact %s verify %s" % (
                name, j["config"]["config"], j["value"], j["ms_per_step"] * 1e3, r["kernel_avg_us"], r["frac"],
                j["bit_exact_vs_reference"], v.get("kernel_avg_us")))
        elif "variants" in j:
            print("%-22s %s" % (name, {k: v.get("median_us", v.get("us")) for k, v in j["variants"].items()}))
