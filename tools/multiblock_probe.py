#!/usr/bin/env python3
"""DIAGNOSTIC: many HDFS blocks in separate device buffers, checksummed one
launch per block (a config-3 plan run on each buffer) vs one launch for all
of them (a CRC32C_DEVICE_ADDRESSES plan over every block's packets).  Per-
block GPU time, steady state, rotating over two sets of buffers; results
checked equal.

    python tools/multiblock_probe.py [--blocks 16] [--iters 200]
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
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import load_package

    hdfs = load_package()
    from hdfs_crc32c_amd.workloads import uniform_packets

    dev = torch.device("cuda", 0)
    nb = args.blocks
    block = uniform_packets(64)  # one 4 MiB block of 64 KiB packets
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    sets = [[torch.randint(0, 256, (4 << 20,), dtype=torch.uint8, device=dev, generator=g) for _ in range(nb)]
            for _ in range(2)]
    ctx = hdfs.Context(0)
    per_block = ctx.plan(block)
    multi = []
    for bufs in sets:
        rows = []
        for k, b in enumerate(bufs):
            pk = block.copy()
            pk["payload_off"] += np.uint64(b.data_ptr())
            pk["out_idx"] += np.uint64(k * 8192)
            rows.append(pk)
        multi.append(hdfs.Plan(ctx, np.concatenate(rows), hdfs.CRC32C_DEVICE_ADDRESSES))
    outs = [torch.zeros(nb * 8192, dtype=torch.int32, device=dev) for _ in range(2)]
    s = torch.cuda.current_stream()

    def one_per_block(i):
        bufs, out = sets[i % 2], outs[i % 2]
        for k in range(nb):
            per_block.exec(bufs[k].data_ptr(), out.data_ptr() + 4 * k * 8192, s.cuda_stream)

    def one_launch(i):
        multi[i % 2].exec(0, outs[i % 2].data_ptr(), s.cuda_stream)

    one_per_block(0)
    torch.cuda.synchronize()
    ref = outs[0].clone()
    outs[0].zero_()
    one_launch(0)
    torch.cuda.synchronize()
    exact = bool(torch.equal(ref, outs[0]))

    def timed(fn):
        for i in range(20):
            fn(i)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for i in range(args.iters):
            fn(i)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (args.iters * nb)

    res = {"per_block_launches": [], "one_launch": []}
    for _ in range(args.rounds):
        res["per_block_launches"].append(timed(one_per_block))
        res["one_launch"].append(timed(one_launch))
    out = {"blocks": nb, "block_bytes": 4 << 20, "exact": exact}
    for k, v in res.items():
        v = sorted(v)
        out[k] = {"us_per_block_median": round(v[len(v) // 2], 3),
                  "GB_s": round((4 << 20) / (v[len(v) // 2] * 1e-6) / 1e9, 1)}
    print(json.dumps(out))
    for p in multi:
        p.close()
    per_block.close()
    ctx.close()


if __name__ == "__main__":
    main()
