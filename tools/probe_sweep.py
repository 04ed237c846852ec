#!/usr/bin/env python3
"""DIAGNOSTIC: sweep plain HBM read shapes (stream_probe.hip) over a config-2
sized buffer (256 MiB, 4 rotating buffers) to find the read pattern the chip
serves fastest; the CRC kernel's roofline fraction is priced against it.

    python tools/probe_sweep.py [--iters 20] [--rounds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {  # shape id -> (name, grids)
    7: ("gs256_u1_nt", (512, 1024, 2048)),
    4: ("gs256_u2_nt", (256, 512, 1024, 2048)),
    2: ("gs256_u4_nt", (256, 512, 768, 1024)),
    5: ("gs256_u8_nt", (256, 512, 768, 1024)),
    6: ("gs256_u16_nt", (256, 512)),
    0: ("gs256_u4", (512,)),
    8: ("t1024_8k_range", (256, 512)),
    9: ("t1024_8k_stride", (256, 512)),
    10: ("t1024_4k_range", (256, 512)),
    11: ("t1024_4k_stride", (256, 512)),
    12: ("t512_8k_range", (256, 512, 1024)),
    13: ("t512_8k_stride", (256, 512, 1024)),
    14: ("t512_4k_range", (256, 512, 1024)),
    15: ("t512_4k_stride", (256, 512, 1024)),
    16: ("t1024_8k_dyn1", (256,)),
    17: ("t1024_8k_static1", (256,)),
    18: ("t1024_8k_dyn4", (256,)),
    19: ("t1024_8k_static4", (256,)),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--nbuf", type=int, default=4)
    ap.add_argument("--shapes", default="", help="comma-separated shape ids (default: all)")
    args = ap.parse_args()
    import torch

    from bench import load_package

    hdfs = load_package()
    L = hdfs.lib()
    extent = 256 << 20
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    bufs = [torch.randint(0, 256, (extent,), dtype=torch.uint8, device=dev, generator=g) for _ in range(args.nbuf)]
    out = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    res = {}
    for r in range(args.rounds):
        for shape, (name, grids) in SHAPES.items():
            if args.shapes and str(shape) not in args.shapes.split(","):
                continue
            for grid in grids:
                def go(i):
                    rc = L.crc32c_debug_stream_probe(bufs[i % args.nbuf].data_ptr(), extent, out.data_ptr(), grid, shape,
                                                     stream.cuda_stream)
                    if rc:
                        raise SystemExit("probe shape %d grid %d: rc %d" % (shape, grid, rc))
                for i in range(2):
                    go(i)
                e0.record(stream)
                for i in range(args.iters):
                    go(i)
                e1.record(stream)
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / args.iters * 1e3
                key = "%s_g%d" % (name, grid)
                res[key] = min(res.get(key, 1e9), us)
    table = {k: {"us": round(v, 2), "TBps": round(extent / (v * 1e-6) / 1e12, 3)} for k, v in sorted(res.items(), key=lambda kv: kv[1])}
    print(json.dumps({"bytes": extent, "probes": table}, indent=0))


if __name__ == "__main__":
    main()
