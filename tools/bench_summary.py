#!/usr/bin/env python3
"""One line per bench.py JSON line found in the given log files (a GPU
session's step logs): config, kernel µs, roofline fraction, value, verify,
and the default line's config4 / strong_scaling sub-objects.

    python tools/bench_summary.py gpurun_out/r5g/*.log
"""
from __future__ import annotations

import json
import sys


def main():
    for fn in sys.argv[1:]:
        try:
            lines = [ln for ln in open(fn) if ln.startswith("{") and '"metric"' in ln]
        except OSError:
            continue
        for ln in lines:
            d = json.loads(ln)
            rf = d.get("roofline") or {}
            v = d.get("verify") or {}
            out = {"log": fn.split("/")[-1], "config": (d.get("config") or {}).get("config"), "n": d.get("n_gpus"),
                   "steps": d.get("steps"), "kernel_us": rf.get("kernel_avg_us"), "frac": rf.get("frac"),
                   "value": d.get("value"), "ms_per_step": d.get("ms_per_step"),
                   "exact": d.get("bit_exact_vs_reference"), "verify_us": v.get("kernel_avg_us"),
                   "verify_graph_us": v.get("graph_kernel_avg_us"), "launch": d.get("launch")}
            c4 = d.get("config4")
            if c4:
                out["c4"] = {k: c4.get(k) for k in ("kernel_step_us", "frac_of_hbm_roofline", "shard_kernel_us",
                                                    "gather_us", "gib_s", "bit_exact", "launch")}
            st = d.get("strong_scaling")
            if st:
                out["strong"] = {k: st.get(k) for k in ("kernel_us_max_rank", "gib_s", "bit_exact")}
            if d.get("cpu_baseline"):
                out["cpu"] = d["cpu_baseline"].get("value")
            print(json.dumps(out))


if __name__ == "__main__":
    main()
