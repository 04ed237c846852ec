#!/usr/bin/env python3
"""FETCH_SIZE per launch of tools/write_probe.py's three plans, from a
rocprofv3 --pmc FETCH_SIZE --kernel-trace output directory.  The CRC
kernel's dispatches come in plan order (zero, data, fuse4), `launches`
each.  FETCH_SIZE is KiB of HBM reads; x2 for gfx950's wide-stream
under-count (MI355X_MICROARCH.md), reported both ways.

    python tools/write_probe_summary.py gpurun_out/wpmc [--launches 23] [--out profiles/...json]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--launches", type=int, default=23)
    ap.add_argument("--out")
    args = ap.parse_args()
    rows = defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(args.pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "hdfs_crc32c_plan_kernel" not in r["Kernel_Name"] or r["Counter_Name"] != "FETCH_SIZE":
                    continue
                d = int(r["Dispatch_Id"])
                rows[d] += float(r["Counter_Value"])
                names[d] = r["Kernel_Name"]
    ids = sorted(rows)
    res = {}
    for k, plan in enumerate(("zero", "data", "fuse4")):
        sel = ids[k * args.launches:(k + 1) * args.launches]
        if not sel:
            continue
        steady = sel[3:] or sel  # after the warm-up launches
        kib = sum(rows[d] for d in steady) / len(steady)
        res[plan] = {"fetch_kib_per_launch": round(kib, 1), "hbm_read_bytes_x2": int(kib * 1024 * 2),
                     "kernel": names[sel[0]], "dispatches": len(sel)}
    res["payload_bytes_per_launch"] = 4 << 20
    text = json.dumps(res, indent=1)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
