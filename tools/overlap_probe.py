#!/usr/bin/env python3
"""DIAGNOSTIC: does a launch's fixed cost (table staging, the CU end-time
tail, the kernel boundary) disappear when independent batches are launched
on S streams, so that the next batch's workgroups start on CUs the previous
one has released?  Config-2 batches over NBUF rotating buffers, one plan
per stream, S = 1 vs 2 (vs 3) interleaved over rounds, steady state (a long
warm-up first: DESIGN.md section 5).

    python tools/overlap_probe.py [--rounds 5] [--iters 1000] [--warmup 500]
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--nbuf", type=int, default=4)
    ap.add_argument("--streams", default="1,2,3")
    ap.add_argument("--config", default="c2")
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import load_package

    hdfs = load_package()
    from hdfs_crc32c_amd.workloads import config_packets

    pk, _ = config_packets(args.config)
    nbytes = int(pk["len"].astype(np.int64).sum())
    extent = int((pk["payload_off"] + pk["len"]).max())
    nout = hdfs.total_checksums(pk)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    bufs = [torch.randint(0, 256, (extent,), dtype=torch.uint8, device=dev, generator=g) for _ in range(args.nbuf)]
    outs = [torch.zeros(nout, dtype=torch.int32, device=dev) for _ in range(args.nbuf)]
    ctx = hdfs.Context(0)
    counts = [int(s) for s in args.streams.split(",")]
    smax = max(counts)
    streams = [torch.cuda.Stream(device=dev) for _ in range(smax)]
    plans = [hdfs.Plan(ctx, pk) for _ in range(smax)]
    main_s = torch.cuda.current_stream()

    def run(nst, iters):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(main_s)
        for s in streams[:nst]:
            s.wait_event(e0)
        for i in range(iters):
            k = i % nst
            b = i % args.nbuf
            plans[k].exec(bufs[b].data_ptr(), outs[b].data_ptr(), streams[k].cuda_stream)
        for s in streams[:nst]:
            ev = torch.cuda.Event()
            ev.record(s)
            main_s.wait_event(ev)
        e1.record(main_s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / iters

    run(1, args.warmup)
    res = {n: [] for n in counts}
    for _ in range(args.rounds):
        for n in counts:
            run(n, 50)
            res[n].append(run(n, args.iters))
    # every buffer's checksums must still be exact (compare with a 1-stream pass)
    ref = [o.clone() for o in outs]
    run(1, args.nbuf)
    torch.cuda.synchronize()
    exact = all(torch.equal(a, b) for a, b in zip(ref, outs))
    table = {}
    for n, t in res.items():
        t = sorted(t)
        med = t[len(t) // 2]
        table["streams_%d" % n] = {"us_per_batch_median": round(med, 2), "us_min": round(t[0], 2),
                                   "TBps_median": round(nbytes / (med * 1e-6) / 1e12, 3)}
    print(json.dumps({"config": args.config, "bytes": nbytes, "exact": exact, "results": table}))
    for p in plans:
        p.close()
    ctx.close()


if __name__ == "__main__":
    main()
