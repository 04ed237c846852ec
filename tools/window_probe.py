#!/usr/bin/env python3
"""Where the bench's wall-clock window loses time beside its kernels
("How the bench times it").

bench.py's value is bytes / the host's clock around K steps; with K = 20
(the driver's command) ~24 us of the window are not kernel time.  This
times, on one GPU, the host-side pieces of that window:

  sync_idle_us       -- torch.cuda.synchronize() with nothing queued;
  record_spin_us     -- event record, then spin on event.query() until done
                        (the host -> GPU -> host round trip of one command);
  record_sync_us     -- event record, then torch.cuda.synchronize();
  launch_sync_us     -- one config-2 launch + synchronize, minus the kernel's
                        own event-timed duration (launch path + completion);
  launch_spin_us     -- the same, completion seen by spinning on an event;
  k20_sync / k20_spin -- bench-like windows of 20 launches (4 host-issued +
                        a graph of 16) ended by synchronize / by an event
                        spin, host clock per step, beside the GPU window;
  lead_pos_us / graph16_us_per_step -- GPU time of each of the four
                        host-issued lead steps (events between them) and
                        per step of the graph of 16 after them;
  ab_host16 / ab_graph16 -- after 4 host-issued steps, 16 more host-issued
                        back to back against the graph of 16 (interleaved).

Prints one JSON line."""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import bench

    hdfs = bench.load_package()
    hdfs.lib()
    from hdfs_crc32c_amd.workloads import synthetic_bytes, uniform_packets

    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    pk = uniform_packets(4096)
    nbytes = 4096 * 65536
    bufs = [torch.from_numpy(synthetic_bytes(nbytes, 7 + b)).to(dev) for b in range(2)]
    outs = [torch.zeros(4096 * 128, dtype=torch.int32, device=dev) for _ in range(2)]
    ctx = hdfs.Context(0)
    plan = ctx.plan(pk)

    def step(i, s=None):
        plan.exec(bufs[i % 2].data_ptr(), outs[i % 2].data_ptr(), sptr if s is None else s)

    res = {}

    def med(xs):
        return round(float(np.median(xs)), 2)

    torch.cuda.synchronize()
    xs = []
    for _ in range(200):
        t = time.perf_counter()
        torch.cuda.synchronize()
        xs.append((time.perf_counter() - t) * 1e6)
    res["sync_idle_us"] = med(xs)
    for mode in ("spin", "sync"):
        xs = []
        for _ in range(200):
            e = torch.cuda.Event()
            t = time.perf_counter()
            e.record(stream)
            if mode == "spin":
                while not e.query():
                    pass
            else:
                torch.cuda.synchronize()
            xs.append((time.perf_counter() - t) * 1e6)
        res["record_%s_us" % mode] = med(xs)
    for i in range(300):  # warm + settle
        step(i)
    torch.cuda.synchronize()
    for mode in ("spin", "sync"):
        xs, ks = [], []
        for i in range(100):
            for j in range(20):  # keep the clocks where they are in a run
                step(j)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            t = time.perf_counter()
            e0.record(stream)
            step(i)
            e1.record(stream)
            if mode == "spin":
                while not e1.query():
                    pass
            torch.cuda.synchronize()
            xs.append((time.perf_counter() - t) * 1e6)
            ks.append(e0.elapsed_time(e1) * 1e3)
        res["launch_%s_us" % mode] = med(xs)
        res["launch_%s_kernel_us" % mode] = med(ks)
        res["launch_%s_overhead_us" % mode] = round(med(xs) - med(ks), 2)
    # bench-like windows
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cs = torch.cuda.current_stream(dev).cuda_stream
        for i in range(4, 20):
            step(i, cs)
    g.replay()
    torch.cuda.synchronize()
    for mode in ("sync", "spin"):
        hs, ws = [], []
        for rep in range(30):
            for i in range(200):
                step(i)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            t = time.perf_counter()
            e0.record(stream)
            for i in range(4):
                step(i)
            g.replay()
            e1.record(stream)
            if mode == "spin":
                while not e1.query():
                    pass
            torch.cuda.synchronize()
            hs.append((time.perf_counter() - t) * 1e6 / 20)
            ws.append(e0.elapsed_time(e1) * 1e3 / 20)
        res["k20_%s_host_us_per_step" % mode] = med(hs)
        res["k20_%s_gpu_us_per_step" % mode] = med(ws)
        res["k20_%s_gap_us_total" % mode] = round((med(hs) - med(ws)) * 20, 2)
    # per-position GPU time inside a bench-like window: events between the
    # four host-issued lead launches, then the graph of 16
    pos = [[] for _ in range(6)]
    for rep in range(30):
        for i in range(200):
            step(i)
        torch.cuda.synchronize()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        evs[0].record(stream)
        for i in range(4):
            step(i)
            evs[i + 1].record(stream)
        g.replay()
        evs[5].record(stream)
        torch.cuda.synchronize()
        for k in range(4):
            pos[k].append(evs[k].elapsed_time(evs[k + 1]) * 1e3)
        pos[5].append(evs[4].elapsed_time(evs[5]) * 1e3 / 16)
    res["lead_pos_us"] = [med(pos[k]) for k in range(4)]
    res["graph16_us_per_step"] = med(pos[5])
    # 16 steps host-issued back to back against the graph of 16, after the
    # same 4 host-issued steps, interleaved (per step, GPU time)
    ab = {"host16": [], "graph16": []}
    for rep in range(40):
        for mode in ("host16", "graph16") if rep % 2 else ("graph16", "host16"):
            for i in range(200):
                step(i)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            for i in range(4):
                step(i)
            e0.record(stream)
            if mode == "graph16":
                g.replay()
            else:
                for i in range(4, 20):
                    step(i)
            e1.record(stream)
            torch.cuda.synchronize()
            ab[mode].append(e0.elapsed_time(e1) * 1e3 / 16)
    res["ab_host16_us_per_step"] = med(ab["host16"])
    res["ab_graph16_us_per_step"] = med(ab["graph16"])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
