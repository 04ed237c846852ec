#!/usr/bin/env python3
"""DIAGNOSTIC: per-launch GPU time of crc32c_plan_exec launched one by one on
a stream vs the same launches captured once into a HIP graph (stream
capture through torch.cuda.CUDAGraph, i.e. hipStreamBeginCapture) and
replayed.  Small batches are launch-bound (a 4 MiB block takes ~5 us, an
empty-ish kernel ~3.5 us back to back), so this measures what a graph saves.

    python tools/graph_probe.py [--config c3] [--per-graph 100] [--rounds 5] [--op exec|verify]
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
    ap.add_argument("--config", default="c3")
    ap.add_argument("--per-graph", type=int, default=100)
    ap.add_argument("--replays", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--nbuf", type=int, default=4)
    ap.add_argument("--op", default="exec", choices=["exec", "verify"])
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
    g.manual_seed(9)
    bufs = [torch.randint(0, 256, (extent,), dtype=torch.uint8, device=dev, generator=g) for _ in range(args.nbuf)]
    outs = [torch.zeros(nout, dtype=torch.int32, device=dev) for _ in range(args.nbuf)]
    ctx = hdfs.Context(0)
    plan = hdfs.Plan(ctx, pk)
    s = torch.cuda.Stream(device=dev)
    K = args.per_graph

    res_buf = torch.zeros(2, dtype=torch.int32, device=dev)

    def launches(stream, op="exec"):
        for i in range(K):
            b = i % args.nbuf
            if op == "exec":
                plan.exec(bufs[b].data_ptr(), outs[b].data_ptr(), stream.cuda_stream)
            else:  # (expected = the checksums the exec launches left in outs)
                plan.verify(bufs[b].data_ptr(), outs[b].data_ptr(), res_buf.data_ptr(), stream.cuda_stream)

    # reference checksums (plain launches), then clear and check the graph's
    with torch.cuda.stream(s):
        launches(s)
    torch.cuda.synchronize()
    ref = [o.clone() for o in outs]
    graph = torch.cuda.CUDAGraph()
    if args.op == "verify":
        with torch.cuda.stream(s):
            launches(s, "verify")  # (the plan's verify stream is now s: no cross-stream wait in the capture)
        torch.cuda.synchronize()
    with torch.cuda.graph(graph, stream=s):
        launches(torch.cuda.current_stream(), args.op)
    if args.op == "exec":
        for o in outs:
            o.zero_()
    graph.replay()
    torch.cuda.synchronize()
    exact = all(torch.equal(a, b) for a, b in zip(ref, outs))
    if args.op == "verify":
        exact = exact and res_buf.cpu().tolist() == [0, -1]

    def timed(fn):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            fn()  # warm
            e0.record(s)
            for _ in range(args.replays):
                fn()
            e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (args.replays * K)

    res = {"stream": [], "graph": []}
    for _ in range(args.rounds):
        res["stream"].append(timed(lambda: launches(s, args.op)))
        res["graph"].append(timed(graph.replay))
    out = {"config": args.config, "op": args.op, "bytes": nbytes, "launches_per_graph": K, "graph_exact": exact}
    for k, v in res.items():
        v = sorted(v)
        out[k] = {"us_per_launch_median": round(v[len(v) // 2], 3), "us_min": round(v[0], 3),
                  "GBps_median": round(nbytes / (v[len(v) // 2] * 1e-6) / 1e9, 1)}
    print(json.dumps(out))
    plan.close()
    ctx.close()


if __name__ == "__main__":
    main()
