#!/usr/bin/env python3
"""Diagnostic: per-launch time of small batches, host-issued vs graph-replayed.

For each config: back-to-back plan.exec launches issued from Python (and the
host's own issue time per launch), then the same launches captured in a graph
of 100 and replayed, for the production kernel and the debug library's
variants given.  Then a plain read kernel (debug stream probe, 512 x 256
threads, no LDS) over the same byte counts: the launch floor of a kernel that
only streams its input.

    python tools/launch_probe.py [--configs c3,p16,p256] [--variants 52]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,p16,p256")
    ap.add_argument("--variants", default="52")
    ap.add_argument("--no-read-probe", action="store_true")
    args = ap.parse_args()
    import torch

    from bench import load_package

    h = load_package()
    from hdfs_crc32c_amd.workloads import config_packets

    variants = [int(v) for v in args.variants.split(",") if v]
    res = {}
    G, R = 100, 20

    def graph_time(s, launch):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for i in range(G):
                launch(i)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(R):
            g.replay()
        e1.record(s)
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / (R * G) * 1e3, 2)

    for cfg in args.configs.split(","):
        pk, _ = config_packets(cfg)
        extent = int((pk["payload_off"] + pk["len"]).max())
        n = h.total_checksums(pk)
        ctx = h.Context(0)
        plan = ctx.plan(pk)
        bufs = [torch.randint(0, 256, (extent,), dtype=torch.uint8, device="cuda") for _ in range(4)]
        outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(4)]
        s = torch.cuda.Stream()
        K = 2000
        r = {"tiles": int(h.debug_plan(pk)[0].size)}
        with torch.cuda.stream(s):
            for i in range(200):
                plan.exec(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
            t0 = time.perf_counter()
            for i in range(K):
                plan.exec(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), s.cuda_stream)
            t1 = time.perf_counter()
            e1.record(s)
            torch.cuda.synchronize()
            r["python_loop_us"] = round(e0.elapsed_time(e1) / K * 1e3, 2)
            r["host_issue_us"] = round((t1 - t0) / K * 1e6, 2)
            r["graph_us"] = graph_time(s, lambda i: plan.exec(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(),
                                                              s.cuda_stream))
            for v in variants:
                r["graph_us_variant%d" % v] = graph_time(
                    s, lambda i, v=v: plan.exec_variant(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), v, 0,
                                                        s.cuda_stream))
        res[cfg] = r
        print(cfg, r, flush=True)
        plan.close()
        ctx.close()

    if not args.no_read_probe:
        L = h.debug_lib()
        for cfg, nbytes in (("4MiB", 4 << 20), ("1MiB", 1 << 20), ("16MiB", 16 << 20), ("64KiB", 1 << 16)):
            src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
            dst = torch.zeros(1 << 20, dtype=torch.int32, device="cuda")
            s = torch.cuda.Stream()

            def probe(i):
                rc = L.crc32c_debug_stream_probe(src.data_ptr(), nbytes, dst.data_ptr(), 512, 2, s.cuda_stream)
                if rc:
                    raise RuntimeError("stream probe rc %d" % rc)

            with torch.cuda.stream(s):
                for i in range(200):
                    probe(i)
                torch.cuda.synchronize()
                res["read_probe_" + cfg] = {"graph_us": graph_time(s, probe), "bytes": nbytes}
            print(cfg, res["read_probe_" + cfg], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
