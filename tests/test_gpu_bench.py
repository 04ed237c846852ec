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
    sys.path.insert(0, ROOT)
    import bench

    assert bench.line_problems(d, want_cpu=False) == [] and d["cpu_baseline"] is None  # (--no-cpu)
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
    # the other two shapes of the 1/2/4/8-GPU curve ride on the default line
    c4 = d["config4"]
    assert c4["bit_exact"] is True and c4["mode"] == "rccl" and c4["n_ranks"] == 1
    assert c4["bit_exact_checks"]["before_warmup_file0"] is True and all(c4["bit_exact_checks"].values())
    assert c4["kernel_step_us"] > 0 and c4["gib_s"] > 0 and c4["shard_kernel_us"] > 0
    assert "hip graph" in c4["launch"] and c4["communicator_rebuilt"] == 0 and c4["transfers"] == 0
    st = d["strong_scaling"]
    assert st["bit_exact"] is True and st["n_ranks"] == 1 and st["packets_per_rank"] == 4096
    assert st["gib_s"] > 0 and 0 < st["frac_of_hbm_roofline_per_gpu"] < 1


def test_bench_injected_capture_failure_falls_back_and_rebuilds():
    """BENCH_CAPTURE_FAIL_RANK=0 at N = 1, config 4 through RCCL (self-send):
    the step capture fails, the communicator is rebuilt, the steps are issued
    from the host and the gathered file is still bit-exact."""
    env = dict(os.environ, BENCH_CAPTURE_FAIL_RANK="0", BENCH_C4_SELF_SEND="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c4", "--steps", "20",
                        "--warmup", "5", "--no-cpu", "--nbuf", "2", "--settle-ms", "20"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    c4 = _line(r.stdout)["config4"]
    assert c4["bit_exact"] is True and c4["self_send"] is True and c4["transfers"] == 1
    assert c4["communicator_rebuilt"] == 1 and c4["launch"].startswith("host-issued")
    assert "injected" in c4["launch"]


@pytest.mark.parametrize("config", ["c2", "c5"])
def test_bench_two_ranks_rehearsal(config):
    """N = 2 (gloo rehearsal): the line is complete at N > 1 -- node-level
    roofline fields and, on c2, the reference CPU baseline timed on rank 0
    after both ranks' GPU work (c5 runs with --no-cpu)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", BENCH_DIST_BACKEND="gloo")
    port = 29500 + random.randrange(2000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "20", "--warmup", "5", "--config", config, "--nbuf", "2"]
    cmd += ["--cpu-seconds", "0.3"] if config == "c2" else ["--no-cpu"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = _line(r.stdout)
    sys.path.insert(0, ROOT)
    import bench

    assert bench.line_problems(d, want_cpu=config == "c2") == []
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["roofline"]["peak_node"] == 16000.0 and 0 < d["roofline"]["frac_node"] < 1
    assert d["bit_exact_vs_reference"] is True  # MIN over ranks, host-resident runs included
    assert d["host_resident_ranks"] == 2 and d["host_resident_gib_s"] > 0
    assert d["gather_ms"] is not None
    if config == "c2":
        assert d["cpu_baseline"]["kind"] == "reference" and d["cpu_baseline"]["value"] > 0
    else:
        assert d["cpu_baseline"] is None
    assert d["config"]["payload_bytes_per_rank"] > 0
    if config == "c2":  # the sub-objects at N = 2 (config 4 as a gloo rehearsal: ranks share the GPU)
        c4 = d["config4"]
        assert c4["n_ranks"] == 2 and c4["bit_exact"] is True and c4["mode"].startswith("gloo rehearsal")
        assert c4["transfers"] == 16 and all(c4["bit_exact_checks"].values())
        st = d["strong_scaling"]
        assert st["n_ranks"] == 2 and st["packets_per_rank"] == 2048 and st["bit_exact"] is True
    else:
        assert d["config4"] is None and d["strong_scaling"] is None


def test_bench_config4_line_two_ranks_complete():
    """`--config c4` at N = 2 (gloo rehearsal): the c4 main line also carries
    the reference CPU baseline and the node-level roofline fields."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", BENCH_DIST_BACKEND="gloo")
    port = 29500 + random.randrange(2000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "10", "--warmup", "2", "--config", "c4", "--nbuf", "2", "--cpu-seconds", "0.3"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = _line(r.stdout)
    sys.path.insert(0, ROOT)
    import bench

    assert bench.line_problems(d) == []
    assert d["n_gpus"] == 2 and d["bit_exact_vs_reference"] is True and d["cpu_baseline"]["kind"] == "reference"
    assert d["roofline"]["frac_node"] == pytest.approx(d["roofline"]["frac"], abs=2e-4)  # (c4's step bytes are the whole file's)


def test_bench_two_ranks_capture_failure_on_one_rank():
    """A graph-capture failure on rank 1 only: both ranks issue from the host
    (the MIN-agreed fallback), and the line is still bit-exact."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", BENCH_DIST_BACKEND="gloo", BENCH_CAPTURE_FAIL_RANK="1")
    port = 29500 + random.randrange(2000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "20", "--warmup", "5", "--no-cpu", "--no-host", "--nbuf", "2", "--no-config4"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["bit_exact_vs_reference"] is True
    assert d["launch"].startswith("host-issued") and "another rank" in d["launch"]  # rank 0 captured, yet fell back
    assert d["strong_scaling"]["launch"].startswith("host-issued")


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
