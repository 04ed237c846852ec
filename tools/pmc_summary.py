#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (tools/pmc_session.sh output) for the CRC32C
kernel: per-dispatch average of every counter, kernel duration, derived HBM
bytes (MI355X_MICROARCH.md HBM section: FETCH_SIZE is in KiB and on gfx950
reads 1/2 of a wide coalesced stream's bytes -> x2; WRITE_SIZE exact), clock
and LDS utilisation.

    python tools/pmc_summary.py gpurun_out/pmc [--out profiles/r01_pmc_c2.json] [--config c2]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

KERNEL = "hdfs_crc32c_plan_kernel"


def load(pmc_dir: str):
    per = defaultdict(lambda: defaultdict(list))  # counter -> dispatch -> values
    durations = {}
    meta = {}
    for f in glob.glob(os.path.join(pmc_dir, "*", "p_counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if KERNEL not in row["Kernel_Name"]:
                    continue
                key = (os.path.basename(os.path.dirname(f)), row["Dispatch_Id"])
                per[row["Counter_Name"]][key].append(float(row["Counter_Value"]))
                durations[key] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                meta = {k: row[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                            "VGPR_Count", "SGPR_Count", "Scratch_Size")}
    out = {}
    for c, d in per.items():
        vals = [sum(v) for v in d.values()]
        out[c] = sum(vals) / len(vals)
    dur = sorted(durations.values())
    return out, dur, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--out")
    ap.add_argument("--config", default="c2")
    ap.add_argument("--bytes", type=int, default=268435456, help="algorithmic bytes per launch")
    args = ap.parse_args()
    c, dur, meta = load(args.pmc_dir)
    med_ns = dur[len(dur) // 2] if dur else None
    import subprocess
    try:  # the commit the profiled library was built from (collect right after committing)
        commit = subprocess.run(["git", "describe", "--always", "--dirty"], capture_output=True, text=True,
                                cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))).stdout.strip()
    except Exception:
        commit = None
    res = {"kernel": KERNEL, "config": args.config, "counters_avg_per_dispatch": c, "dispatch_meta": meta,
           "profiled_duration_ns_median": med_ns, "commit": commit}
    if "FETCH_SIZE" in c:
        fetch = c["FETCH_SIZE"] * 1024 * 2  # KiB; gfx950 under-count of wide streams corrected x2
        write = c.get("WRITE_SIZE", 0.0) * 1024
        res["hbm_read_bytes_per_launch"] = fetch
        res["hbm_write_bytes_per_launch"] = write
        res["hbm_bytes_per_launch"] = fetch + write
        res["traffic_over_algorithmic"] = (fetch + write) / args.bytes
    if "GRBM_GUI_ACTIVE" in c and med_ns:
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md DVFS item)
        res["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / med_ns
    if "SQ_LDS_IDX_ACTIVE" in c and "GRBM_GUI_ACTIVE" in c:
        res["lds_busy_frac_per_cu"] = c["SQ_LDS_IDX_ACTIVE"] / (c["GRBM_GUI_ACTIVE"] / 8 * 256)
    if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c:
        res["lds_bank_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1)
    text = json.dumps(res, indent=1, sort_keys=True)
    print(text)
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
