#!/usr/bin/env python3
"""Per-launch durations of one kernel from a rocprofv3 kernel trace
(run_kernel_trace.csv), averaged over bench.py's timed window: launch 0 is
the correctness gate, then `--estimate` launches that time one step (round
4), then (graph-replayed bench, the default) one untimed replay of the
captured launches -- the `--steps` minus a host-issued lead of `--lead`
(round 4: the line's `kernel_timing` names it) --, then `--settle`
power-settle launches (the line's `settle_launches`), then `--warmup`
warm-up launches, then the `--steps` timed ones, of which the bench times
the kernel over those after the lead.  Writes the window's average / median / min / max (ns) so it can be
compared with bench.py's own HIP-event average for the same run.

    python tools/trace_window.py gpurun_out/prof/run_kernel_trace.csv \
        --kernel "hdfs_crc32c_plan_kernel<768, 3, 3>" [--warmup 500 --steps 2000] [--out f.json]
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--settle", type=int, default=0, help="the bench line's settle_launches")
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--out")
    ap.add_argument("--no-graph", action="store_true", help="the bench ran with --no-graph (no untimed replay)")
    ap.add_argument("--estimate", type=int, default=10, help="step-time estimate launches (round 4 bench)")
    ap.add_argument("--lead", type=int, default=0, help="host-issued lead steps (not captured)")
    args = ap.parse_args()
    rows = [r for r in csv.DictReader(open(args.trace)) if args.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    pre = 1 + args.estimate + (0 if args.no_graph else args.steps - args.lead)
    first = pre + args.settle + args.warmup + args.lead
    nwin = args.steps - args.lead
    win = dur[first:first + nwin]
    starts = [int(r["Start_Timestamp"]) for r in rows[first:first + nwin]]
    res = {
        "kernel": args.kernel, "launches_in_trace": len(dur), "window": [first, first + len(win)],
        "window_avg_ns": round(statistics.mean(win), 1), "window_median_ns": statistics.median(win),
        "window_min_ns": min(win), "window_max_ns": max(win),
        "window_span_per_launch_ns": round((starts[-1] - starts[0]) / max(len(starts) - 1, 1), 1),
        "settle_avg_ns": round(statistics.mean(dur[pre:pre + args.settle]), 1) if args.settle else None,
        "warmup_avg_ns": round(statistics.mean(dur[pre + args.settle:pre + args.settle + args.warmup]), 1)
        if args.warmup else None,
    }
    text = json.dumps(res, indent=1)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
