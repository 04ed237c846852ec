#!/usr/bin/env python3
"""DIAGNOSTIC: where the host-resident path (crc32c_batch_host) loses against
a plain pinned H2D copy.  Times batch_host and a torch pinned->device copy of
the same bytes at several batch sizes (fixed vs per-byte cost), with the
output array preallocated, interleaved over rounds.

    python tools/host_probe.py [--rounds 5] [--reps 5] [--packets 1024,4096,16384]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--packets", default="1024,4096,16384")
    ap.add_argument("--pageable", action="store_true", help="batch_host from pageable memory (CPU staging copy)")
    ap.add_argument("--shuffle-blocks", action="store_true",
                    help="packets in 4 MiB blocks taken in a shuffled order (scattered pinned runs)")
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import load_package

    hdfs = load_package()
    from hdfs_crc32c_amd.workloads import synthetic_bytes, uniform_packets

    ctx = hdfs.Context(0)
    dev = torch.device("cuda", 0)
    sizes = [int(x) for x in args.packets.split(",")]
    big = max(sizes) * 65536
    pinned = torch.empty(big, dtype=torch.uint8).pin_memory()
    pinned.numpy()[:] = synthetic_bytes(big, 11)
    hp = pinned.numpy().copy() if args.pageable else pinned.numpy()
    dst = torch.empty(big, dtype=torch.uint8, device=dev)
    res = {}
    def packets(n):
        pk = uniform_packets(n)
        if args.shuffle_blocks and n >= 64:
            perm = np.random.default_rng(n).permutation(n // 64)
            pk = pk.reshape(-1, 64)[perm].reshape(-1).copy()
            pk["out_idx"] = np.arange(n, dtype=np.uint64) * 128
        return pk

    for n in sizes:  # warm: staging buffers, plans
        pk = packets(n)
        out = np.zeros(hdfs.total_checksums(pk), np.uint32)
        ctx.batch_host(hp, pk, out=out)
        dst[: n * 65536].copy_(pinned[: n * 65536], non_blocking=True)
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for n in sizes:
            nb = n * 65536
            pk = packets(n)
            out = np.zeros(hdfs.total_checksums(pk), np.uint32)
            t0 = time.perf_counter()
            for _ in range(args.reps):
                ctx.batch_host(hp, pk, out=out)
            t_host = (time.perf_counter() - t0) / args.reps
            t0 = time.perf_counter()
            for _ in range(args.reps):
                dst[:nb].copy_(pinned[:nb], non_blocking=True)
            torch.cuda.synchronize()
            t_copy = (time.perf_counter() - t0) / args.reps
            r = res.setdefault(n, {"host_ms": 1e9, "copy_ms": 1e9})
            r["host_ms"] = min(r["host_ms"], t_host * 1e3)
            r["copy_ms"] = min(r["copy_ms"], t_copy * 1e3)
    for n, r in res.items():
        nb = n * 65536
        r["host_gib_s"] = round(nb / (r["host_ms"] * 1e-3) / GIB, 2)
        r["copy_gib_s"] = round(nb / (r["copy_ms"] * 1e-3) / GIB, 2)
        r["host_ms"] = round(r["host_ms"], 3)
        r["copy_ms"] = round(r["copy_ms"], 3)
    print(json.dumps({"slice_mb": os.environ.get("HDFS_CRC32C_SLICE_MB", "default"),
                      "shuffled_blocks": args.shuffle_blocks, "pageable": args.pageable, "sizes": res}))
    ctx.close()


if __name__ == "__main__":
    main()
