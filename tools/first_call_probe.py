#!/usr/bin/env python3
"""A process's first checksum calls (a FUSE daemon's first block write):
host time of crc32c_ctx_create, then of the first three exec + synchronise
round trips of a one-block plan (config 3: one 4 MiB block), then the
median of 50 more.  Run in a fresh process each time (the first launch of a
code object loads it).  Prints one JSON line."""
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
    pk = uniform_packets(64)
    buf = torch.from_numpy(synthetic_bytes(64 * 65536, 3)).to(dev)
    out = torch.zeros(64 * 128, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter()
    ctx = hdfs.Context(0)
    res = {"ctx_create_ms": round((time.perf_counter() - t) * 1e3, 3)}
    plan = ctx.plan(pk)
    s = torch.cuda.current_stream(dev)
    xs = []
    for i in range(53):
        t = time.perf_counter()
        plan.exec(buf.data_ptr(), out.data_ptr(), s.cuda_stream)
        s.synchronize()
        xs.append((time.perf_counter() - t) * 1e6)
    res["first_calls_us"] = [round(x, 1) for x in xs[:3]]
    res["steady_call_us"] = round(float(np.median(xs[3:])), 1)
    print(json.dumps(res))
    plan.close()
    ctx.close()


if __name__ == "__main__":
    main()
