#!/usr/bin/env python3
"""DIAGNOSTIC: per-wave stamps of the scheduler-wave kernel (variant 30: 8 u64
per wave: start, staged, end, hw ids, then for workers {ring pops, ticks
waiting on the ring} and for the scheduler {grabs, summed grab round trip,
longest grab, first grab time}).  Ticks are s_memrealtime (100 MHz)."""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import oracle
    from bench import config_packets, load_package

    variant = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    wpg = int(sys.argv[2]) if len(sys.argv) > 2 else 13
    hdfs = load_package()
    pk, _ = config_packets("c2", oracle)
    extent = int((pk["payload_off"] + pk["len"]).max())
    nout = hdfs.total_checksums(pk)
    dev = torch.device("cuda", 0)
    bufs = [torch.randint(0, 256, (extent,), dtype=torch.uint8, device=dev) for _ in range(4)]
    out = torch.zeros(nout, dtype=torch.int32, device=dev)
    os.environ["HDFS_CRC32C_KVARIANT"] = "0"
    ctx = hdfs.Context(0)
    plan = ctx.plan(pk)
    stamps = torch.zeros(8 * 256 * wpg, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    q = lambda a: [round(float(np.percentile(a, x)), 2) for x in (0, 10, 50, 90, 100)]
    runs = []
    for rep in range(3):
        for b in range(3):
            plan.exec(bufs[b].data_ptr(), out.data_ptr(), s)
        stamps.zero_()
        plan.exec_variant(bufs[3].data_ptr(), out.data_ptr(), variant, stamps.data_ptr(), s)
        torch.cuda.synchronize()
        st = stamps.cpu().numpy().reshape(-1, 8)
        used = st[:, 0] != 0
        idx = np.flatnonzero(used)
        st = st[used]
        t0 = st[:, 0].min()
        end = (st[:, 2] - t0) / 100.0
        is_sched = (idx % wpg) == (wpg - 1)
        wk, sc = st[~is_sched], st[is_sched]
        runs.append({
            "span_us": round(float(end.max()), 2),
            "worker_end_us": q(end[~is_sched]),
            "worker_pops": q(wk[:, 4]), "worker_ring_wait_us": q(wk[:, 5] / 100.0),
            "sched_grabs": q(sc[:, 4]), "sched_grab_rt_avg_us": q(sc[:, 5] / np.maximum(sc[:, 4], 1) / 100.0),
            "sched_grab_rt_max_us": q(sc[:, 6] / 100.0),
            "sched_first_grab_us": q((sc[:, 7] - t0) / 100.0 * (sc[:, 7] > 0)),
            "sched_end_us": q(end[is_sched]),
        })
    print(json.dumps({"variant": variant, "runs": runs}, indent=1))


if __name__ == "__main__":
    main()
