#!/usr/bin/env python3
"""Diagnostic: per-wave timeline of the CRC32C kernel from the stamped
variant (s_memrealtime, 100 MHz).  Prints start/staging/end distributions
(us, relative to the first wave start) overall and per XCD.  Stamps are only
in the diagnostic build's buffer; read the SHARES, not the length."""
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

    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    variant = int(sys.argv[2]) if len(sys.argv) > 2 else 5  # 5 = production + stamps, 6 = memory-only + stamps
    wpg = int(sys.argv[3]) if len(sys.argv) > 3 else 12  # waves per workgroup of that variant
    hdfs = load_package()
    from hdfs_crc32c_amd.workloads import config_packets

    pk, _ = config_packets(cfg)
    extent = int((pk["payload_off"] + pk["len"]).max())
    nout = hdfs.total_checksums(pk)
    dev = torch.device("cuda", 0)
    bufs = [torch.randint(0, 256, (extent,), dtype=torch.uint8, device=dev) for _ in range(4)]
    out = torch.zeros(nout, dtype=torch.int32, device=dev)
    # (the plan is the production one; stamped variants run through the debug library)
    ctx = hdfs.Context(0)
    plan = ctx.plan(pk)
    stamps = torch.zeros(4 * 256 * 2 * 16, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    res = []
    # placement: which CU / XCD each workgroup ran on (from run 0)
    placement = None
    cu_ends = []  # per run: {cu key: last end}
    wg_ends = []  # per run: per-workgroup last end, by blockIdx
    for rep in range(4):
        for b in range(3):
            plan.exec(bufs[b].data_ptr(), out.data_ptr(), s)
        stamps.zero_()
        plan.exec_variant(bufs[3].data_ptr(), out.data_ptr(), variant, stamps.data_ptr(), s)
        torch.cuda.synchronize()
        st = stamps.cpu().numpy().reshape(-1, 4)
        st = st[st[:, 0] != 0]
        t0 = st[:, 0].min()
        start = (st[:, 0] - t0) / 100.0
        staged = (st[:, 1] - t0) / 100.0
        end = (st[:, 2] - t0) / 100.0
        xcc = (st[:, 3] >> 32) & 0xF
        q = lambda a: [round(float(np.percentile(a, x)), 2) for x in (0, 10, 50, 90, 100)]
        wg = np.arange(st.shape[0]) // wpg
        # HW_ID: cu_id [11:8], sh_id [12], se_id [15:13]; tg_id [19:16] is the
        # workgroup slot on the CU and must not split one CU into several.
        cu = (xcc << 16) | (((st[:, 3] & 0xFFFFFFFF) >> 8) & 0xFF)
        wg_end = {}
        wg_cu = {}
        for w in np.unique(wg):
            m = wg == w
            wg_end[int(w)] = (float(end[m].min()), float(end[m].max()))
            wg_cu[int(w)] = int(cu[m][0])
        spread_in_wg = [b - a for a, b in wg_end.values()]
        by_cu = {}
        for w, c in wg_cu.items():
            by_cu.setdefault(c, []).append(wg_end[w][1])
        pair_gap = [max(v) - min(v) for v in by_cu.values() if len(v) == 2]
        cu_ends.append({c: max(v) for c, v in by_cu.items()})
        if placement is None:
            placement = [wg_cu[w] for w in sorted(wg_cu)]
        wg_ends.append(np.array([wg_end[w][1] for w in sorted(wg_end)]))
        res.append({
            "wg_end_spread_us_pct": q(np.array(spread_in_wg)),
            "cu_pair_end_gap_us_pct": q(np.array(pair_gap)) if pair_gap else None,
            "wgs_per_cu": sorted(set(len(v) for v in by_cu.values())),
            "cu_last_end_us_pct": q(np.array([max(v) for v in by_cu.values()])),
            "waves": int(st.shape[0]), "span_us": round(float(end.max()), 2),
            "start_us_pct": q(start), "staging_us_pct": q(staged - start), "work_us_pct": q(end - staged),
            "end_us_pct": q(end),
            "per_xcd_end_max": [round(float(end[xcc == x].max()), 2) if np.any(xcc == x) else None for x in range(8)],
            "per_xcd_waves": [int(np.sum(xcc == x)) for x in range(8)],
            "xcc_of_block_0_to_7": [int(xcc[wg == b][0]) if np.any(wg == b) else None for b in range(8)],
            "group_mean_end": [round(float(np.mean([wg_end[w][1] for w in wg_end if w % 8 == g])), 2) for g in range(8)],
        })
    # Is a slow CU slow in every run (a property of the CU) or at random?
    keys = sorted(set.intersection(*[set(d) for d in cu_ends]))
    m = np.array([[d[k] for k in keys] for d in cu_ends])
    cc = np.corrcoef(m)
    wcc = np.corrcoef(np.array([w for w in wg_ends if len(w) == len(wg_ends[0])]))
    xcd_of = np.array([k >> 16 for k in keys])
    extra = {"cu_end_corr_between_runs": [round(float(x), 3) for x in cc[np.triu_indices(len(cc), 1)]],
             "wg_end_corr_between_runs": [round(float(x), 3) for x in wcc[np.triu_indices(len(wcc), 1)]],
             "cu_mean_end_by_xcd": [round(float(m[:, xcd_of == x].mean()), 2) for x in range(8)],
             "wg_end_by_blockidx_mod8": [round(float(np.mean([w[i::8].mean() for w in wg_ends])), 2) for i in range(8)],
             "placement_first_40": [hex(c) for c in placement[:40]],
             "placement_256_280": [hex(c) for c in placement[256:280]],
             "wg_end_by_blockidx_decile": [round(float(np.mean([w[i * len(w) // 10:(i + 1) * len(w) // 10].mean() for w in wg_ends])), 2) for i in range(10)]}
    print(json.dumps({"config": cfg, "variant": variant, "runs": res, "analysis": extra}, indent=1))


if __name__ == "__main__":
    main()
