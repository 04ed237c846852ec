#!/usr/bin/env python3
"""A/B of a launch's fixed cost, graph-replayed,
interleaved rounds on one box:

  c2         -- config 2: one plan over 4096 x 64 KiB packets, one launch per step
  c2_halves  -- the same batch as two half-plans, the second on a forked
                stream joined back by events inside the step (its workgroups
                start on the CUs the first half's tail frees)
  c4         -- config 4 at N = 1: one plan over the 128 MiB file (what
                crc32c_multi_plan_exec launches in place)
  c4_blocks  -- the same file as ONE crc32c_plan_exec_blocks launch of a
                one-block plan over 32 block pointers
  c4_halves  -- the file as two half-plans on forked streams

Every mode rotates over 4 distinct payloads (no Infinity-Cache reuse) and
checks its last step's checksums against the reference after timing.

    python tools/fixed_cost_probe.py [--rounds 3] [--steps 2000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import load_package, reference_checksums  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--modes", default="c2,c2_halves,c4,c4_blocks,c4_halves")
    args = ap.parse_args()
    import torch

    hdfs = load_package()
    hdfs.lib()
    from hdfs_crc32c_amd.workloads import synthetic_bytes, uniform_packets

    dev = torch.device("cuda", 0)
    ctx = hdfs.Context(0)
    main_s = torch.cuda.Stream(device=dev)
    side_s = torch.cuda.Stream(device=dev)
    nbuf = 4
    modes = {}

    def batch(npk, seed):
        pk = uniform_packets(npk)
        host = synthetic_bytes(npk * 65536, seed)
        bufs = [torch.from_numpy(host).to(dev)] + [torch.randint(0, 256, (npk * 65536,), dtype=torch.uint8,
                                                                 device=dev) for _ in range(nbuf - 1)]
        outs = [torch.zeros(npk * 128, dtype=torch.int32, device=dev) for _ in range(nbuf)]
        return pk, host, bufs, outs

    def whole(npk, seed):
        pk, host, bufs, outs = batch(npk, seed)
        plan = ctx.plan(pk)

        def step(i, s):
            plan.exec(bufs[i % nbuf].data_ptr(), outs[i % nbuf].data_ptr(), s)
        return step, (pk, host, outs[0]), npk * 65536

    def halves(npk, seed):
        pk, host, bufs, outs = batch(npk, seed)
        h = npk // 2
        pa = ctx.plan(pk[:h])
        pb_pk = pk[h:].copy()
        pb_pk["payload_off"] -= pb_pk["payload_off"][0]
        pb_pk["out_idx"] -= pb_pk["out_idx"][0]
        pb = ctx.plan(pb_pk)
        off_b, oidx_b = h * 65536, h * 128

        def step(i, s):
            b = i % nbuf
            side_s.wait_stream(torch.cuda.current_stream(dev))
            pa.exec(bufs[b].data_ptr(), outs[b].data_ptr(), s)
            pb.exec(bufs[b].data_ptr() + off_b, outs[b].data_ptr() + 4 * oidx_b, side_s)
            torch.cuda.current_stream(dev).wait_stream(side_s)
        return step, (pk, host, outs[0]), npk * 65536

    def blocks32(seed):
        pk, host, bufs, outs = batch(2048, seed)
        plan = ctx.plan(uniform_packets(64))

        def step(i, s):
            b = i % nbuf
            plan.exec_blocks([bufs[b].data_ptr() + k * (4 << 20) for k in range(32)],
                             [outs[b].data_ptr() + 4 * k * 8192 for k in range(32)], s)
        return step, (pk, host, outs[0]), 2048 * 65536

    for name in args.modes.split(","):
        if name == "c2":
            modes[name] = whole(4096, 11)
        elif name == "c2_halves":
            modes[name] = halves(4096, 12)
        elif name == "c4":
            modes[name] = whole(2048, 13)
        elif name == "c4_blocks":
            modes[name] = blocks32(14)
        elif name == "c4_halves":
            modes[name] = halves(2048, 15)

    graphs = {}
    torch.cuda.synchronize()
    for name, (step, _, _) in modes.items():
        with torch.cuda.stream(main_s):
            for i in range(nbuf):  # (plans' first launch on the capture stream outside the capture)
                step(i, main_s.cuda_stream)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=main_s, capture_error_mode="thread_local"):
            for i in range(args.steps):
                step(i, main_s.cuda_stream)
        graphs[name] = g
        for out in modes[name][1][2:]:
            out.zero_()
    torch.cuda.synchronize()
    res = {n: [] for n in modes}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(args.rounds):
        for name, g in graphs.items():
            with torch.cuda.stream(main_s):  # (a graph replays on the current stream)
                g.replay()  # (settle: the package runs at its power cap after ~0.1 s)
                e0.record(main_s)
                g.replay()
                e1.record(main_s)
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / args.steps)
            print(json.dumps({"round": r, "mode": name, "us_per_step": round(res[name][-1], 3)}), flush=True)
    out = {}
    for name, (step, (pk, host, out0), nbytes) in modes.items():
        want = reference_checksums(host, pk, pk.size * 128)
        exact = bool(np.array_equal(out0.cpu().numpy().view(np.uint32), want))
        us = float(np.median(res[name]))
        out[name] = {"us_per_step_median": round(us, 3), "runs": [round(x, 3) for x in res[name]],
                     "frac_of_8TBs": round(nbytes / (us * 1e-6) / 8e12, 4), "bit_exact": exact}
    print(json.dumps({"summary": out}), flush=True)


if __name__ == "__main__":
    main()
