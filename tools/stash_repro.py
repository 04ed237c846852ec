#!/usr/bin/env python3
"""Diagnostic (round 3): the verify-only miscompare of the
abandoned tail-row templating build (git stash@{0}).  Runs the batch of
tests/test_general_tiles_any_bpc against ONE library build given on the
command line (scratch/<build>/: a copy of the package's __init__.py and the
libhdfs_crc32c.so built from that tree), exec + verify + verify_bitmap, a few
repeats, and prints one JSON line per bpc: exec exact?, verify counts,
where the mismatches are (chunk index mod 16 = the item lane, item numbers),
and -- for the diagnostic build whose kernel records (computed, expected) of
every mismatch through HDFS_DIAG_REC -- whether the computed value or the
fetched expected value was the wrong one.  The oracle is the checker."""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(build_dir: str):
    spec = importlib.util.spec_from_file_location("hdfs_build", os.path.join(build_dir, "__init__.py"),
                                                  submodule_search_locations=[build_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["hdfs_build"] = mod
    spec.loader.exec_module(mod)
    mod.lib()
    return mod


def batch(hdfs, bpc):  # tests/test_gpu_write_read.py test_general_tiles_any_bpc
    rows, off, out = [], 0, 0
    tails = [4, 5, 100, 508, 509, 511, 513, 1000, 1023, 1025, 4097]
    for i in range(20):
        ln = 65536 - (0 if i % 3 else 777)
        if i % 3 == 2:
            ln = 65536 // bpc * bpc - bpc + tails[i % len(tails)] % bpc
        rows.append((off, out, ln, bpc))
        out += (ln + bpc - 1) // bpc
        off += ln + (i % 16) + 1
    return np.array(rows, hdfs.PACKET_DTYPE), off, out


def main():
    import torch

    import oracle

    build = sys.argv[1]
    bpcs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [4]
    hdfs = load(os.path.join(ROOT, "scratch", build))
    orc = oracle.Oracle()
    ctx = hdfs.Context(0)
    stream = torch.cuda.current_stream()
    for bpc in bpcs:
        pk, off, nout = batch(hdfs, bpc)
        payload = oracle.xorshift64_bytes(off + 64, 3000 + bpc)
        payload[:bpc * 2] = 0
        want = orc.batch(payload, pk, nout)
        dev = torch.from_numpy(payload).cuda()
        plan = hdfs.Plan(ctx, pk)
        out = torch.full((nout,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        plan.exec(dev.data_ptr(), out.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        exec_exact = bool(np.array_equal(out.cpu().numpy().view(np.uint32), want))
        exp = torch.from_numpy(want.view(np.int32).copy()).cuda()
        rec = torch.zeros(nout, dtype=torch.int64, device="cuda")
        os.environ["HDFS_DIAG_REC"] = str(rec.data_ptr())  # (read only by the diagnostic build)
        runs = []
        bad_sets = []
        for rep in range(4):
            res = torch.zeros(2, dtype=torch.int32, device="cuda")
            bits = torch.zeros((nout + 31) // 32, dtype=torch.int32, device="cuda")
            plan.verify(dev.data_ptr(), exp.data_ptr(), res.data_ptr(), stream.cuda_stream,
                        dev_bad_bits=bits.data_ptr() if rep % 2 else 0)
            torch.cuda.synchronize()
            r = res.cpu().numpy().view(np.uint32).tolist()
            runs.append(r)
            if rep % 2:
                flags = np.unpackbits(bits.cpu().numpy().view(np.uint8), bitorder="little")[:nout]
                bad_sets.append(np.flatnonzero(flags))
        del os.environ["HDFS_DIAG_REC"]
        line = {"build": build, "bpc": bpc, "nout": nout, "exec_exact": exec_exact, "verify_runs": runs}
        tiles, gen = hdfs.debug_plan(pk)
        line["items"] = {"tiles": int(tiles.size), "gen": int(gen.size)}
        if bad_sets:
            b = bad_sets[-1]
            line["bitmap_bad"] = int(b.size)
            line["bitmap_same_each_run"] = all(np.array_equal(b, x) for x in bad_sets)
            if b.size:
                # which item: the tile whose out range holds the index
                starts = tiles["out"].astype(np.int64)
                order = np.argsort(starts)
                pos = np.searchsorted(starts[order], b, side="right") - 1
                item = order[np.clip(pos, 0, None)]
                lane = b - starts[item]
                line["bad_first"] = b[:12].tolist()
                line["bad_lane_hist"] = np.bincount(np.clip(lane, 0, 16), minlength=17).tolist()
                line["bad_items"] = int(np.unique(item).size)
                line["bad_items_first"] = np.unique(item)[:12].tolist()
                metas = tiles["meta"][np.unique(item)]
                line["bad_item_nch"] = np.unique((metas >> 13) & 31).tolist()
                line["bad_item_tail"] = np.unique(tiles["src"][np.unique(item)] >> np.uint64(48)).tolist()
                line["all_items_nch_hist"] = np.bincount((tiles["meta"] >> 13) & 31, minlength=17).tolist()
                recs = rec.cpu().numpy().view(np.uint64)[b]
                if recs.any():
                    got = (recs >> np.uint64(32)).astype(np.uint32)
                    expd = (recs & np.uint64(0xFFFFFFFF)).astype(np.uint32)
                    line["rec_computed_right"] = int(np.sum(got == want[b]))
                    line["rec_expected_right"] = int(np.sum(expd == want[b]))
                    line["rec_samples"] = [["%08x" % g, "%08x" % e, "%08x" % w] for g, e, w in
                                           zip(got[:6], expd[:6], want[b][:6])]
        print(json.dumps(line), flush=True)
        plan.close()
    ctx.close()


if __name__ == "__main__":
    main()
