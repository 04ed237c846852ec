#!/usr/bin/env python3
"""Workload for PMC passes over the packet-assembly plans
(crc32c_plan_create_buffers): N launches each of
  zero  -- a 4 MiB ftruncate extension, one NULL buffer (fuse.c:1137-1142):
           every checksum is a plan-time constant, nothing should be read;
  data  -- the same 4 MiB from one device buffer (tiles);
  fuse4 -- TRUNCATE / NULLPADDING / THEDATA / TRAILINGDATA buffers
           (fuse.c:1348-1354) summing to 4 MiB.
Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace -- python3 tools/write_probe.py`;
tools/write_probe_summary.py attributes the dispatches (in this order) and
prints FETCH_SIZE per launch.  Also prints the per-launch time of each.
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from bench import load_package

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    hdfs = load_package()
    hdfs.lib()
    ctx = hdfs.Context(0)
    mb4 = 4 << 20
    data = torch.randint(0, 256, (mb4 + 64,), dtype=torch.uint8, device="cuda")
    base = data.data_ptr()
    plans = {
        "zero": ctx.write_plan([(0, mb4)], 0, mb4),
        "data": ctx.write_plan([(base, mb4)], 0, mb4),
        "fuse4": ctx.write_plan([(base, 100000), (0, 300000), (base + 400000, 3000000),
                                 (base + 3400000 + 17, mb4 - 3400000)], 0, mb4),
    }
    out = torch.zeros(8192 + 64, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    res = {}
    for name, plan in plans.items():
        for _ in range(3):
            plan.exec(0, out.data_ptr(), s.cuda_stream)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(n):
            plan.exec(0, out.data_ptr(), s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        res[name] = {"us_per_launch": round(e0.elapsed_time(e1) / n * 1e3, 2), "launches": n + 3}
    if np.any(out[:8192].cpu().numpy().view(np.uint32) == 0):
        raise SystemExit("unexpected zero checksum")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
