#!/usr/bin/env python3
"""Diagnostic: sustained kernel time, package power and shader clock per
kernel variant.  For each variant, ~1.5 s of back-to-back launches is queued
on the stream; rocm-smi is sampled while they run; the average launch time
comes from HIP events around the whole burst.

    python tools/power_probe.py [--variants 0,3,4] [--launches 30000]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def smi():
    try:
        out = subprocess.run(["rocm-smi", "--showpower", "--showclocks"], capture_output=True, text=True,
                             timeout=20).stdout
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)}
    pw = re.findall(r"Package Power \(W\): ([0-9.]+)", out)
    sclk = re.findall(r"sclk clock level: \S+ \((\d+)Mhz\)", out)
    return {"power_w": float(pw[0]) if pw else None, "sclk_mhz": int(sclk[0]) if sclk else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,3,4")
    ap.add_argument("--launches", type=int, default=30000)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--external-smi", action="store_true", help="power is sampled by tools/power_probe.sh")
    args = ap.parse_args()
    import torch

    from bench import load_package

    hdfs = load_package()
    from hdfs_crc32c_amd.workloads import config_packets

    pk, _ = config_packets(args.config)
    nbytes = int(pk["len"].astype("int64").sum())
    extent = int((pk["payload_off"] + pk["len"]).max())
    nout = hdfs.total_checksums(pk)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    bufs = [torch.randint(0, 256, (extent,), dtype=torch.uint8, device=dev, generator=g) for _ in range(4)]
    outs = [torch.zeros(nout, dtype=torch.int32, device=dev) for _ in range(4)]
    s = torch.cuda.current_stream()
    res = {}
    for v in args.variants.split(","):
        ctx = hdfs.Context(0)
        plan = ctx.plan(pk)

        def launch(i, v=int(v)):  # variant 0: the product entry; others: the debug library
            if v == 0:
                plan.exec(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), s.cuda_stream)
            else:
                plan.exec_variant(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), v, 0, s.cuda_stream)

        for i in range(20):
            launch(i)
        torch.cuda.synchronize()
        time.sleep(1.0)  # let clocks / power settle back
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        t_begin = time.time()
        e0.record(s)
        for i in range(args.launches):
            launch(i)
        e1.record(s)
        samples = [] if args.external_smi else [smi() for _ in range(2)]
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / args.launches * 1e3
        res[v] = {"us_per_launch": round(us, 2), "GBps": round(nbytes / (us * 1e-6) / 1e9, 1), "smi": samples,
                  "wall": [round(t_begin, 2), round(time.time(), 2)]}
        plan.close()
        ctx.close()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
