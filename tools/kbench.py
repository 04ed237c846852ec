#!/usr/bin/env python3
"""A/B timing of the kernel variants in ONE process, interleaved rounds
(cdna_hip_programming.md 5.4 rule 24).  Device-resident config-2 batches
rotating over NBUF buffers; reports per-variant median/min kernel time and
GB/s, and checks every variant's checksums against variant 0.

    python tools/kbench.py [--rounds 7] [--iters 20] [--config c2|c5|c3|pN]
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--nbuf", type=int, default=4)
    ap.add_argument("--variants", default="0,1,2,3,4,5")
    ap.add_argument("--verify", action="store_true", help="also time crc32c_plan_verify (production) as 'verify_0'")
    args = ap.parse_args()

    import numpy as np
    import torch

    from bench import load_package

    hdfs = load_package()
    from hdfs_crc32c_amd.workloads import config_packets

    pk, workload = config_packets(args.config)  # c2 / c3 / c5, or pN: N uniform 64 KiB packets
    nbytes = int(pk["len"].astype(np.int64).sum())
    extent = int((pk["payload_off"] + pk["len"]).max())
    nout = hdfs.total_checksums(pk)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    bufs = [torch.randint(0, 256, (extent,), dtype=torch.uint8, device=dev, generator=g) for _ in range(args.nbuf)]
    outs = [torch.zeros(nout, dtype=torch.int32, device=dev) for _ in range(args.nbuf)]
    variants = args.variants.split(",")
    # One plan; variant 0 through the product entry point (crc32c_plan_exec),
    # the others through the debug library's crc32c_debug_plan_exec_variant.
    ctx = hdfs.Context(0)
    the_plan = ctx.plan(pk)
    stream = torch.cuda.current_stream()

    class _Runner:
        def __init__(self, v):
            self.v = int(v)

        def exec(self, src, dst, s):
            if self.v == 0:
                the_plan.exec(src, dst, s)
            else:
                the_plan.exec_variant(src, dst, self.v, 0, s)

        def verify(self, *a):
            the_plan.verify(*a)

    plans = {v: (ctx, _Runner(v)) for v in variants}
    ref = None
    for v in variants:
        plans[v][1].exec(bufs[0].data_ptr(), outs[0].data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        got = outs[0].cpu().numpy().copy()
        if ref is None:
            ref = got
        if not np.array_equal(got, ref):
            print("note: variant %s checksums differ (diagnostic variant?)" % v, file=sys.stderr)
    times = {v: [] for v in variants}
    vvars = [v for v in variants if int(v) == 0] if args.verify else []  # the production compare mode
    if vvars:
        exps = [torch.zeros_like(o) for o in outs]
        for i in range(args.nbuf):  # expected checksums of every buffer (diagnostic variants overwrite outs)
            plans[vvars[0]][1].exec(bufs[i].data_ptr(), exps[i].data_ptr(), stream.cuda_stream)
        vres = torch.zeros(2, dtype=torch.int32, device=dev)
        for v in vvars:
            times["verify_" + v] = []
    for r in range(args.rounds):
        for v in vvars:
            vplan = plans[v][1]
            for i in range(3):
                vplan.verify(bufs[i % args.nbuf].data_ptr(), exps[i % args.nbuf].data_ptr(), vres.data_ptr(),
                             stream.cuda_stream)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(args.iters):
                b = i % args.nbuf
                vplan.verify(bufs[b].data_ptr(), exps[b].data_ptr(), vres.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            times["verify_" + v].append(e0.elapsed_time(e1) / args.iters * 1e3)
            assert vres.cpu().tolist() == [0, -1], vres
        for v in variants:
            plan = plans[v][1]
            for i in range(3):
                plan.exec(bufs[i % args.nbuf].data_ptr(), outs[i % args.nbuf].data_ptr(), stream.cuda_stream)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(args.iters):
                b = i % args.nbuf
                plan.exec(bufs[b].data_ptr(), outs[b].data_ptr(), stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.iters * 1e3)  # us per launch
    # reference: device-to-device copy of one buffer (read + write bytes)
    dst = torch.empty_like(bufs[0])
    for _ in range(3):
        dst.copy_(bufs[1])
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(args.iters):
        dst.copy_(bufs[i % args.nbuf])
    e1.record(stream)
    torch.cuda.synchronize()
    copy_us = e0.elapsed_time(e1) / args.iters * 1e3
    res = {"torch_copy": {"us": round(copy_us, 2), "GBps_rw": round(2 * extent / (copy_us * 1e-6) / 1e9, 1)}}
    # reference: plain streaming reads (stream_probe.hip), several shapes
    probe_out = torch.zeros(256 * 256 * 16, dtype=torch.int32, device=dev)
    L = hdfs.debug_lib()
    for shape in (0, 2):
        for grid in (512, 1024):
            tt = []
            for r in range(3):
                for i in range(2):
                    L.crc32c_debug_stream_probe(bufs[i % args.nbuf].data_ptr(), extent, probe_out.data_ptr(), grid, shape,
                                                stream.cuda_stream)
                e0.record(stream)
                for i in range(args.iters):
                    L.crc32c_debug_stream_probe(bufs[i % args.nbuf].data_ptr(), extent, probe_out.data_ptr(), grid,
                                                shape, stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize()
                tt.append(e0.elapsed_time(e1) / args.iters * 1e3)
            res["probe_s%d_g%d" % (shape, grid)] = {"us": round(min(tt), 2),
                                                    "GBps": round(extent / (min(tt) * 1e-6) / 1e9, 1)}
    for v in times:
        t = sorted(times[v])
        res[v] = {"median_us": round(t[len(t) // 2], 2), "min_us": round(t[0], 2),
                  "GBps_median": round(nbytes / (t[len(t) // 2] * 1e-6) / 1e9, 1),
                  "GBps_best": round(nbytes / (t[0] * 1e-6) / 1e9, 1)}
    print(json.dumps({"config": args.config, "workload": workload, "bytes": nbytes, "variants": res}))


if __name__ == "__main__":
    main()
