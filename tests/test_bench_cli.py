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


def test_sub_run_error_is_reported_in_its_sub_object():
    """A sub-run that raises is recorded in its sub-object and the runs after
    it are skipped; the main line is still printed once (publish)."""
    sys.path.insert(0, ROOT)
    import bench

    line = {"metric": "m", "config4": None, "strong_scaling": None}
    wd = bench.SubRunWatchdog(60.0, line)

    def boom():
        raise RuntimeError("rccl init failed")

    bench.line_set(line, "config4", wd.run("config4", boom))
    assert wd.failed and line["config4"] == {"error": "RuntimeError: rccl init failed"}
    assert wd.run("ok", lambda: {"x": 1}) == {"x": 1}
    wd.cancel()


_WATCHDOG_SCRIPT = r"""
import sys, time
sys.path.insert(0, %r)
import bench
line = {"metric": "m", "value": 1.0, "config4": {"kernel_step_us": 24.0}, "strong_scaling": None}
wd = bench.SubRunWatchdog(0.5, line)
wd.start()
wd.run("strong_scaling", time.sleep, 30)
print("not reached")
"""


def test_sub_run_watchdog_prints_the_main_line_and_exits():
    """A hung sub-run (here a sleep standing in for a collective no peer
    joins): past the bound the main line is printed once, with the finished
    sub-object kept and the hung one marked, and the process exits 0."""
    import json

    r = subprocess.run([sys.executable, "-c", _WATCHDOG_SCRIPT % ROOT], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and "not reached" not in r.stdout
    d = json.loads(lines[0])
    assert d["config4"] == {"kernel_step_us": 24.0}
    assert "timed out" in d["strong_scaling"]["error"] and "strong_scaling" in d["strong_scaling"]["error"]
    assert "watchdog fired" in r.stderr
