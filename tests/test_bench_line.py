"""bench.py's line at N > 1 on CPU: the CPU baseline leg runs on rank 0
after every rank's GPU work while the peers wait on the store (gloo, world
size 2 and 3), and the line schema (roofline node fields, cpu_baseline) is
pinned.  The driver's scaling run prints one such line per N = 1/2/4/8."""
from __future__ import annotations

import json
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, out_dir: str):
    from types import SimpleNamespace

    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    import bench
    import oracle

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        env = SimpleNamespace(world=world, rank=rank)
        pk = oracle.uniform_packets(16)
        payload = oracle.xorshift64_bytes(16 * 65536, oracle.SEED)
        calls = []

        def leg():
            calls.append(rank)
            cb = bench.cpu_baseline(pk, payload, 0.05, nbuf=2)
            time.sleep(0.5)  # (the peers must still be waiting after this)
            return cb

        cb = bench.cpu_baseline_on_rank0(env, leg, wait_s=120)
        done = time.time()
        with open(os.path.join(out_dir, "r%d.json" % rank), "w") as f:
            json.dump({"cb": cb, "calls": calls, "done": done}, f)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_cpu_baseline_on_rank0_after_peers_wait(tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [json.load(open(tmp_path / ("r%d.json" % r))) for r in range(world)]
    cb = res[0]["cb"]
    assert res[0]["calls"] == [0] and all(r["calls"] == [] and r["cb"] is None for r in res[1:])
    assert cb["kind"] == "reference" and cb["unit"] == "GiB/s" and cb["value"] > 0 and cb["cores"] >= 1
    assert all(r["done"] >= res[0]["done"] - 0.05 for r in res[1:])  # the peers returned after rank 0's leg


def _line(n: int, frac: float = 0.78) -> dict:
    sys.path.insert(0, ROOT)
    import bench

    nbytes = 268435456
    kus = nbytes / (frac * bench.PEAK_HBM_GBS * 1e9) * 1e6
    return {"metric": "m", "value": 5000.0 * n, "unit": "GiB/s", "n_gpus": n, "steps": 20, "warmup": 5,
            "ms_per_step": 0.0456, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic", "config": {"workload": "c2"},
            "roofline": dict({"bound": "hbm", "achieved": frac * bench.PEAK_HBM_GBS, "peak": bench.PEAK_HBM_GBS,
                              "unit": "GB/s", "frac": frac, "traffic": None}, **bench.roofline_node(nbytes, kus, n)),
            "cpu_baseline": {"value": 353.3, "unit": "GiB/s", "cores": 16, "kind": "reference", "sample": "s"}}


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_line_schema_at_every_n(n):
    import bench

    d = _line(n)
    assert bench.line_problems(d) == []
    rf = d["roofline"]
    # weak scaling: N ranks' bytes over the slowest rank's time against N x 8 TB/s = the per-GPU fraction
    assert rf["peak_node"] == n * 8000.0 and rf["frac_node"] == pytest.approx(0.78, abs=1e-4)
    assert rf["achieved_node"] == pytest.approx(n * 0.78 * 8000.0, rel=1e-3)


def test_line_schema_flags_what_round5_lacked():
    """BENCH_r05's N > 1 form: no cpu_baseline and no node-level roofline."""
    import bench

    d = _line(2)
    d["cpu_baseline"] = None
    for k in ("achieved_node", "peak_node", "frac_node"):
        del d["roofline"][k]
    bad = bench.line_problems(d)
    assert "cpu_baseline is None" in bad and "roofline missing frac_node" in bad
    with open(os.path.join(ROOT, "BENCH_r05.json")) as f:
        r05 = json.load(f)["parsed"]
    assert "roofline missing frac_node" in bench.line_problems(r05)
    assert bench.line_problems(r05, want_cpu=True) == ["roofline missing achieved_node", "roofline missing peak_node",
                                                       "roofline missing frac_node"]
    assert np.isclose(r05["roofline"]["frac"], 0.765)
