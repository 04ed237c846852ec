#!/usr/bin/env python3
"""Summarise a rocprofv3 --memory-copy-trace --kernel-trace run of
tools/host_probe.py (crc32c_batch_host): per-call copy/kernel timeline of the
host-resident pipeline (copy durations, gaps between consecutive H2D copies,
kernel durations, tail from the last copy to the call's last GPU event).

    python tools/copy_trace_summary.py <dir with *_memory_copy_trace.csv> [--out f.json]

Calls are separated by GPU idle gaps > 50 us; the torch reference copies
(one H2D per call of the whole batch) are reported apart.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default="")
    ap.add_argument("--min-copy-mib", type=float, default=1.0, help="H2D copies at least this big are payload")
    args = ap.parse_args()
    mc = glob.glob(os.path.join(args.dir, "**", "*memory_copy_trace.csv"), recursive=True)
    kt = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)
    ev = []
    for r in csv.DictReader(open(mc[0])):
        ev.append({"t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"]), "kind": r["Direction"].replace(
            "MEMORY_COPY_", ""), "stream": r.get("Stream_Id", "")})
    for r in csv.DictReader(open(kt[0])):
        ev.append({"t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"]), "kind": "KERNEL",
                   "name": r["Kernel_Name"], "stream": r.get("Stream_Id", "")})
    ev.sort(key=lambda e: e["t0"])
    # split into bursts separated by idle gaps
    calls, cur, end = [], [], None
    for e in ev:
        if end is not None and e["t0"] - end > 50_000:
            calls.append(cur)
            cur = []
        cur.append(e)
        end = e["t1"] if end is None else max(end, e["t1"])
    if cur:
        calls.append(cur)
    out = {"source": os.path.relpath(mc[0]), "calls": []}
    prev_end = None
    for c in calls:
        idle = None if prev_end is None else round((min(e["t0"] for e in c) - prev_end) / 1e3, 1)
        prev_end = max(e["t1"] for e in c)
        crc = [e for e in c if e["kind"] == "KERNEL" and "crc32c" in e["name"]]
        h2d = [e for e in c if e["kind"] == "HOST_TO_DEVICE"]
        if not crc:  # the torch reference copy
            if h2d:
                out.setdefault("reference_copies_us", []).append(round((h2d[0]["t1"] - h2d[0]["t0"]) / 1e3, 1))
            continue
        span = (max(e["t1"] for e in c) - min(e["t0"] for e in c)) / 1e3
        cd = [(e["t1"] - e["t0"]) / 1e3 for e in h2d]
        gaps = [(b["t0"] - a["t1"]) / 1e3 for a, b in zip(h2d, h2d[1:])]
        last_copy_end = max(e["t1"] for e in h2d) if h2d else min(e["t0"] for e in c)
        out["calls"].append({
            "idle_before_us": idle,
            "span_us": round(span, 1),
            "h2d_copies": len(h2d),
            "h2d_copy_us_mean": round(statistics.mean(cd), 1) if cd else None,
            "h2d_gap_us_mean": round(statistics.mean(gaps), 1) if gaps else None,
            "kernels": len(crc),
            "kernel_us_mean": round(statistics.mean((e["t1"] - e["t0"]) / 1e3 for e in crc), 1),
            "tail_us": round((max(e["t1"] for e in c) - last_copy_end) / 1e3, 1),
            "other_gpu_ops": sorted({e.get("name", e["kind"])[:40] for e in c if e not in crc and e not in h2d}),
        })
    s = json.dumps(out, indent=1)
    print(s)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
