"""bench.py's launch rules on CPU (no GPU call is reached): --gpus N is
honoured or refused, never silently run as one rank."""
from __future__ import annotations

import os
import subprocess
import sys

from conftest import ROOT


def _run(args, **env_over):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "BENCH_DIST_BACKEND"):
        env.pop(k, None)
    env.update(env_over)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=300)


def test_world_size_and_gpus_flag_must_agree():
    r = _run(["--gpus", "2", "--steps", "1"], WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2 and "disagree" in r.stderr, r.stderr[-2000:]
    assert "{" not in r.stdout


def test_gpus_flag_with_rccl_needs_that_many_gpus():
    """Here (no GPU visible) --gpus 2 over RCCL must fail fast, before any
    rank starts, instead of printing an n_gpus: 1 line."""
    import torch

    if torch.cuda.device_count() >= 2:  # (a multi-GPU host would run it for real)
        return
    r = _run(["--gpus", "2", "--steps", "1"])
    assert r.returncode == 2 and "visible GPUs" in r.stderr, r.stderr[-2000:]
    assert "{" not in r.stdout


def test_gpus_flag_must_be_positive():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0 and "--gpus" in r.stderr
