#!/usr/bin/env python3
"""DIAGNOSTIC: why bench.py and tools/kbench.py time the same kernel
differently.  Runs bench.py's exact loop (50 back-to-back launches over 4
rotating 256 MiB buffers, HIP events on the launch stream, then 20 rotating
verify launches) under variations of the setup: buffer 0 host-generated
(xorshift64, as bench.py) or device-generated, and the plan created before
or after the buffers.

    python tools/harness_probe.py [--variant 0] [--reps 3]
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
    ap.add_argument("--variant", default="0")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    from bench import load_package

    hdfs = load_package()  # (production kernel; --variant is kept for old command lines, 0 only)
    assert args.variant == "0", "kernel variants are launched through the debug library (tools/kbench.py)"
    from hdfs_crc32c_amd.workloads import config_packets, synthetic_bytes

    pk, _ = config_packets("c2")
    extent = int((pk["payload_off"] + pk["len"]).max())
    nout = hdfs.total_checksums(pk)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream

    def run(buf0_host: bool, plan_first: bool):
        ctx = plan = None
        if plan_first:
            ctx = hdfs.Context(0)
            plan = ctx.plan(pk)
        g = torch.Generator(device=dev)
        g.manual_seed(1234)
        if buf0_host:
            bufs = [torch.from_numpy(synthetic_bytes(extent, 1)).to(dev)]
        else:
            bufs = [torch.randint(0, 256, (extent,), dtype=torch.uint8, device=dev, generator=g)]
        for _ in range(3):
            bufs.append(torch.randint(0, 256, (extent,), dtype=torch.uint8, device=dev, generator=g))
        outs = [torch.zeros(nout, dtype=torch.int32, device=dev) for _ in range(4)]
        if not plan_first:
            ctx = hdfs.Context(0)
            plan = ctx.plan(pk)
        for i in range(10):
            plan.exec(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), s)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(50):
            plan.exec(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), s)
        e1.record(stream)
        torch.cuda.synchronize()
        ex = e0.elapsed_time(e1) / 50 * 1e3
        res = torch.zeros(2, dtype=torch.int32, device=dev)
        for i in range(3):
            plan.verify(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), res.data_ptr(), s)
        e0.record(stream)
        for i in range(20):
            plan.verify(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), res.data_ptr(), s)
        e1.record(stream)
        torch.cuda.synchronize()
        vf = e0.elapsed_time(e1) / 20 * 1e3
        ok = res.cpu().tolist() == [0, -1]
        plan.close()
        ctx.close()
        del bufs, outs
        torch.cuda.empty_cache()
        return round(ex, 2), round(vf, 2), ok

    out = {}
    for r in range(args.reps):
        for buf0_host in (True, False):
            for plan_first in (True, False):
                key = "buf0_%s_plan_%s" % ("host" if buf0_host else "dev", "first" if plan_first else "last")
                out.setdefault(key, []).append(run(buf0_host, plan_first))
    print(json.dumps({"variant": args.variant, "exec_us_verify_us_ok": out}, indent=1))


if __name__ == "__main__":
    main()
