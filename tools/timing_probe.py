#!/usr/bin/env python3
"""Diagnostic: kernel time of the production plan over a few seconds of
back-to-back launches, in rounds of 20, for buffers filled two ways (the
bench's xorshift64 host stream, and device random bytes).  Shows whether a
run's kernel time depends on how long the GPU has been busy or on the data.

    python tools/timing_probe.py [--seconds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import load_package

    hdfs = load_package()
    from hdfs_crc32c_amd.workloads import synthetic_bytes, uniform_packets

    pk = uniform_packets(4096)
    extent = int((pk["payload_off"] + pk["len"]).max())
    nout = hdfs.total_checksums(pk)
    dev = torch.device("cuda", 0)
    host = torch.from_numpy(synthetic_bytes(extent, 1)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    rnd = [torch.randint(0, 256, (extent,), dtype=torch.uint8, device=dev, generator=g) for _ in range(4)]
    sets = {"xorshift+3rand": [host] + rnd[:3], "4rand": rnd}
    outs = [torch.zeros(nout, dtype=torch.int32, device=dev) for _ in range(4)]
    ctx = hdfs.Context(0)
    plan = ctx.plan(pk)
    s = torch.cuda.current_stream()
    res = {}
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    for name, bufs in list(sets.items()) * 2:
        ts = []
        import time
        t_end = time.perf_counter() + args.seconds / 4
        while time.perf_counter() < t_end:
            e0.record(s)
            for i in range(20):
                plan.exec(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 20 * 1e3)
        q = lambda a, p: round(float(np.percentile(a, p)), 2)
        res.setdefault(name, []).append({"rounds": len(ts), "first5": [round(x, 2) for x in ts[:5]],
                                         "p10": q(ts, 10), "p50": q(ts, 50), "p90": q(ts, 90)})
    # One continuous stream of launches, an event every 25 launches: the
    # kernel time as a function of how long the GPU has been running it.
    n_seg, per = 160, 25
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n_seg + 1)]
    torch.cuda._sleep(1000000)  # ~idle gap before the burst
    torch.cuda.synchronize()
    evs[0].record(s)
    for k in range(n_seg):
        for i in range(per):
            plan.exec(sets["4rand"][i % 4].data_ptr(), outs[i % 4].data_ptr(), s.cuda_stream)
        evs[k + 1].record(s)
    torch.cuda.synchronize()
    seg = [round(evs[k].elapsed_time(evs[k + 1]) / per * 1e3, 1) for k in range(n_seg)]
    res["continuous_us_per_launch_by_25"] = seg
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
