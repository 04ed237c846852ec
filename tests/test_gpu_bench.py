"""bench.py's contract on the GPU, as the driver runs it: one JSON line with
the metric, roofline and correctness fields at N = 1, and the N > 1 path
(torch.distributed launch, barrier, max-over-ranks timing, gather to rank 0,
every rank's host-resident run) rehearsed with two ranks on the one visible
GPU, their collectives over gloo (BENCH_DIST_BACKEND; two RCCL ranks cannot
share one GPU -- the RCCL transport itself is covered by the multi-plan
self-send test).  Short step counts: these check the plumbing, not the rate.
Children are started as subprocesses (never exec'd from this process)."""
from __future__ import annotations

import json
import os
import random
import subprocess
import sys

import pytest

from conftest import ROOT

# (generous limits: on a fresh box the first torch import pages the image in)
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(400)]


@pytest.fixture(scope="module", autouse=True)
def _torch_paged_in():
    import torch  # the children's imports then read a warm page cache

    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"


def _line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out[-3000:]
    return json.loads(lines[-1])


def test_bench_one_gpu_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "200", "--warmup", "20",
                        "--no-cpu", "--no-host"], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and d["steps"] == 200 and d["unit"] == "GiB/s" and d["higher_is_better"]
    assert d["bit_exact_vs_reference"] is True
    # the gate before warm-up, the timed launches on buffer 0 and on a device-random buffer
    assert d["bit_exact_checks"] == {"before_warmup_buf0": True, "timed_buf0": True,
                                     "timed_buf1_device_random": True}
    assert d["verify"]["clean"] is True
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["algorithmic_bytes_per_launch"] == 4096 * 65536
    assert 0 < rf["frac"] < 1 and rf["kernel_avg_us"] > 0
    assert d["value"] > 0 and d["config"]["config"] == "c2"


@pytest.mark.parametrize("config", ["c2", "c5"])
def test_bench_two_ranks_rehearsal(config):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", BENCH_DIST_BACKEND="gloo")
    port = 29500 + random.randrange(2000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "20", "--warmup", "5", "--config", config, "--no-cpu", "--nbuf", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["bit_exact_vs_reference"] is True  # MIN over ranks, host-resident runs included
    assert d["host_resident_ranks"] == 2 and d["host_resident_gib_s"] > 0
    assert d["gather_ms"] is not None and d["cpu_baseline"] is None
    assert d["config"]["payload_bytes_per_rank"] > 0


def test_bench_gpus_flag_spawns_ranks():
    """`python3 bench.py --gpus 2` (the driver's form, no launcher): bench.py
    starts torch.distributed.run with two ranks as a child process and
    forwards rank 0's line -- here rehearsed as two gloo ranks on the one GPU."""
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "c2", "--steps", "20",
                        "--warmup", "5", "--no-cpu", "--nbuf", "2"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["bit_exact_vs_reference"] is True
    assert d["bit_exact_checks"]["timed_buf0"] is True and d["bit_exact_checks"]["timed_buf1_device_random"] is True
    assert len([ln for ln in r.stdout.splitlines() if ln.startswith("{")]) == 1


def test_bench_gpus_flag_refuses_more_rccl_ranks_than_gpus():
    """--gpus N with RCCL needs N GPUs: on a box with fewer it fails fast with
    a message instead of printing an n_gpus: 1 line."""
    import torch

    n = torch.cuda.device_count() + 1
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("BENCH_DIST_BACKEND", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "5"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "visible GPUs" in r.stderr, r.stderr[-2000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
