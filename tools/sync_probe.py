#!/usr/bin/env python3
"""How long the host takes to see a finished launch: wall time of [launch
one config-2 plan exec; torch.cuda.synchronize()] against the kernel's own
event time, median of many, with HIP's default device scheduling or (with
--spin) hipDeviceScheduleSpin set before the device is first used.  Prices
the fixed wall-clock cost around bench.py's timed window.

    python tools/sync_probe.py [--spin] [--reps 200]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spin", action="store_true")
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    import torch

    flags_rc = None
    if args.spin:
        hip = None  # the HIP runtime torch loaded (one per process)
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    hip = ctypes.CDLL(line.split()[-1])
                    break
        flags_rc = hip.hipSetDeviceFlags(ctypes.c_uint(1)) if hip else None  # hipDeviceScheduleSpin
    from bench import load_package

    hdfs = load_package()
    from hdfs_crc32c_amd.workloads import config_packets

    pk, _ = config_packets("c2")
    extent = int((pk["payload_off"] + pk["len"]).max())
    dev = torch.device("cuda", 0)
    buf = torch.randint(0, 256, (extent,), dtype=torch.uint8, device=dev)
    out = torch.zeros(hdfs.total_checksums(pk), dtype=torch.int32, device=dev)
    ctx = hdfs.Context(0)
    plan = ctx.plan(pk)
    s = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(200):
        plan.exec(buf.data_ptr(), out.data_ptr(), s)
    torch.cuda.synchronize()
    walls, kerns, syncs = [], [], []
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        plan.exec(buf.data_ptr(), out.data_ptr(), s)
        e1.record()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        walls.append((t2 - t0) * 1e6)
        syncs.append((t2 - t1) * 1e6)
        kerns.append(e0.elapsed_time(e1) * 1e3)
    print({"spin": args.spin, "set_flags_rc": flags_rc, "wall_us": round(statistics.median(walls), 2),
           "event_window_us": round(statistics.median(kerns), 2),
           "wall_minus_window_us": round(statistics.median(w - k for w, k in zip(walls, kerns)), 2),
           "issue_to_sync_return_us": round(statistics.median(syncs), 2)}, flush=True)


if __name__ == "__main__":
    main()
