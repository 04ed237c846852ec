#!/usr/bin/env python3
"""Bench: device-resident CRC32C over 64 KiB packets x 512 B chunks (BASELINE.json).

One step = one pass of the hot path (hadoop_rpc_send_packet's per-chunk
checksum loop, src/hadooprpc.c:733-742, for a whole batch) over one batch
already resident in HBM: config 2 = 4096 packets x 65536 B = 256 MiB,
bytesPerChecksum 512, 524288 checksums, on every rank (weak scaling: each
GPU checksums its own 256 MiB batch, no data-path collective).  The batch
rotates over NBUF distinct 256 MiB buffers so consecutive steps cannot be
served from the 256 MiB Infinity Cache.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]

N > 1 runs one rank per GPU.  Launched by torch.distributed.run (WORLD_SIZE
set, as the driver does) every process is one rank; launched plainly with
--gpus N > 1 this process starts torch.distributed.run with N ranks as a
child process (before any GPU call; never an exec), forwards its output and
exits with its return code.  After the timed region the ranks' checksum
arrays are gathered to rank 0 over RCCL (the only collective of configs 2/5;
timed separately as "gather_ms"; config 4 gathers inside every step).
Rank 0 prints ONE JSON line.

The default line (config 2, weak scaling) also carries, at every N, the two
other shapes BASELINE.json's 1/2/4/8-GPU curve is quoted on (each timed like
the main steps: K steps, graph-replayed, max over ranks, bit-exact against
the reference):
  config4         -- config 4 (128 MiB file = 32 x 4 MiB blocks dealt
                     round-robin over the ranks, src/fuse.c:580-647): every
                     step is crc32c_multi_plan_exec, the shards' launches AND
                     the RCCL gather of the checksums into file order on
                     rank 0, captured into the step graph;
  strong_scaling  -- the one config-2 batch (256 MiB) split over the ranks.
Graph capture is rank-consistent (native-hdfs-fuse_amd/graphs.py): the
ranks agree (MIN all-reduce) on a probe with no collective and then on the
step capture; if any rank fails, every rank drops its graphs, the config-4
communicator is rebuilt on every rank, and every rank issues its steps from
the host.  BENCH_CAPTURE_FAIL_RANK=r injects a step-capture failure on rank r.
"""
from __future__ import annotations

import argparse
import glob
import importlib.util
import json
import math
import os
import sys
import time
from types import SimpleNamespace

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
KERNEL_NAME = "hdfs_crc32c_plan_kernel"
# Template instance of the production variant on a full batch (crc32c_kernel.hip,
# kVariants[0]: 768 threads, 3 waves/SIMD, kModeS4 | kModeNt); PMC traffic is
# only reported from a summary of this exact kernel.
PRODUCTION_KERNEL = "hdfs_crc32c_plan_kernel<768, 3, 3>"
C4_BLOCKS = 32        # config 4: 128 MiB file = 32 x 4 MiB blocks
C4_GROUP_PACKETS = 64  # one 4 MiB block = 64 packets of 64 KiB
MULTI_SELF_SEND = 0x10  # CRC32C_MULTI_SELF_SEND
MULTI_PIPELINE = 0x40  # CRC32C_MULTI_PIPELINE


def load_package():
    if "hdfs_crc32c_amd" in sys.modules:
        return sys.modules["hdfs_crc32c_amd"]
    pkg_dir = os.path.join(ROOT, "native-hdfs-fuse_amd")
    spec = importlib.util.spec_from_file_location("hdfs_crc32c_amd", os.path.join(pkg_dir, "__init__.py"),
                                                  submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["hdfs_crc32c_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


# ---- the CPU reference leg: the only place bench.py touches oracle/ --------
# The reference's own crc32c.c (oracle/_ref) is the checker of the GPU
# results (outside the timed region) and the timed CPU baseline; nothing it
# computes is measured as or passed off for the product's output.
def reference_checksums(payload: np.ndarray, pk, nout: int) -> np.ndarray:
    """Expected checksums from the reference's crc32c.c (oracle/_ref) when it
    is built, else the clean-room oracle; multi-threaded over packets."""
    import oracle as oracle_mod

    impl = oracle_mod.Reference() if oracle_mod.Reference.available() else oracle_mod.Oracle()
    out = np.zeros(max(nout, 1), np.uint32)
    impl.batch_mt_seconds(payload, pk, out, max(1, min(16, os.cpu_count() or 1)), 1)
    return out[:nout]


def baseline_metric() -> str:
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except Exception:
        return "GiB/s CRC32C, device-resident 64 KiB packets × 512 B chunks, 1/2/4/8 GPU"


def latest_pmc(profile_dir: str, config: str):
    """HBM bytes per launch of the kernel from the newest committed rocprofv3
    PMC summary of this config (profiles/[rNN/[pmc/]]rNN_pmc_<config>.json, written
    by tools/pmc_summary.py)."""
    files = glob.glob(os.path.join(profile_dir, "*pmc_c*.json")) + \
        glob.glob(os.path.join(profile_dir, "r*", "*pmc_c*.json")) + \
        glob.glob(os.path.join(profile_dir, "r*", "pmc", "*pmc_c*.json"))
    best = None
    for fn in sorted(files, key=os.path.basename):
        try:
            with open(fn) as f:
                d = json.load(f)
        except Exception:
            continue
        if d.get("config") == config:
            best = d
    return best


def config_name(name: str) -> str:
    """--config: a BASELINE.json config or one of its variants (c2b<bpc>: config 2 with that bytesPerChecksum;
    c2w<bpc>: the same with packets cut to whole chunks, no tail chunk)."""
    if name in ("c2", "c3", "c4", "c5", "c2u", "c2t", "c3u") or (name[:3] in ("c2b", "c2w") and name[3:].isdigit()
                                                                    and 4 <= int(name[3:]) <= 65536):
        return name
    raise argparse.ArgumentTypeError("unknown config %r" % name)


def cpu_quota():
    """(CPUs this process may run on, CPU bandwidth quota in CPUs or None):
    sched_getaffinity and the cgroup v2 cpu.max / v1 cfs quota -- a container
    can show every host CPU to os.cpu_count() and still cap the time they get."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except Exception:
        affinity = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except Exception:
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = round(q / per, 2)
        except Exception:
            pass
    return affinity, quota


def host_sockets() -> int:
    try:
        with open("/proc/cpuinfo") as f:
            ids = {l.split(":", 1)[1].strip() for l in f if l.startswith("physical id")}
        return max(1, len(ids))
    except Exception:
        return 1


def cpu_baseline(pk, payload_np: np.ndarray, seconds: float, nbuf: int = 4):
    """The reference's own crc32c.c (oracle/_ref, kind "reference") per chunk
    as hadooprpc.c:739-742, on this box's host cores, at full width
    (os.cpu_count() threads), one socket's worth and 1
    thread: each thread owns a contiguous packet slice, the batch is copied
    into `nbuf` distinct first-touched buffers (more than the host L3, as the
    GPU side rotates its buffers) and the passes rotate over them, so the
    rate is a DRAM-streaming one.  Bounded sample: about `seconds` of wall
    time per thread count.  Falls back to the clean-room oracle ("port",
    single-buffer timing) when the reference build is absent."""
    import oracle as oracle_mod

    nout = oracle_mod.total_checksums(pk)
    out = np.zeros(nout, np.uint32)
    nbytes = int(pk["len"].astype(np.int64).sum())
    ncpu = os.cpu_count() or 1
    sockets = host_sockets()
    quota = cpu_quota()[1]
    # full width, one socket, one core -- and, under a cgroup CPU quota, as
    # many threads as the quota's CPUs (more threads than that only share the
    # same CPU time)
    counts = sorted({1, max(1, ncpu // sockets), ncpu} | ({max(1, min(ncpu, int(math.ceil(quota))))} if quota else set()))
    res = {}
    try:
        impl = oracle_mod.Reference()
        kind = "reference"
        for t in counts:
            reps = max(nbuf, 2 * t)
            dt = impl.batch_rot_seconds(payload_np, pk, out, t, nbuf, reps)
            reps = max(nbuf, int(reps * seconds / max(dt, 1e-6)))
            dt = impl.batch_rot_seconds(payload_np, pk, out, t, nbuf, reps)
            res[t] = nbytes * reps / dt / GIB
    except (FileNotFoundError, OSError):
        impl = oracle_mod.Oracle()
        kind = "port"
        for t in counts:
            dt = impl.batch_mt_seconds(payload_np, pk, out, t, 1)
            reps = max(1, int(seconds / max(dt, 1e-6)))
            res[t] = nbytes * reps / impl.batch_mt_seconds(payload_np, pk, out, t, reps) / GIB
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except Exception:
        pass
    # The baseline is the best rate over the thread counts tried (never the
    # understated one): on a box whose cgroup quota lends fewer CPUs' time
    # than it shows, full width oversubscribes that time.
    best = max(res, key=lambda t: res[t])
    return {
        "value": round(res[best], 3), "unit": "GiB/s", "cores": best, "kind": kind,
        "sample": "%s: the config batch (%d packets, %.0f MiB) in %d distinct first-touched host copies rotated "
                  "per pass (DRAM-streaming), ~%.0fs per thread count, best of %s threads; reference crc32c.c "
                  "built -O2 (its Makefile builds -O0)"
                  % (kind, pk.size, nbytes / 2**20, nbuf if kind == "reference" else 1, seconds,
                     "/".join(str(t) for t in counts)),
        "full_width_gib_s": round(res[ncpu], 3),
        "per_threads_gib_s": {str(t): round(v, 3) for t, v in res.items()},
        "one_core_gib_s": round(res[1], 3), "one_socket_gib_s": round(res[max(1, ncpu // sockets)], 3),
        "host_cpus": ncpu, "sockets": sockets, "cpu_model": cpu_model,
        "cpu_affinity": cpu_quota()[0], "cgroup_cpu_quota": cpu_quota()[1],
    }


CPU_BASELINE_KEY = "bench/cpu_baseline_done"


def cpu_baseline_on_rank0(env, fn, wait_s: float = 900.0):
    """The CPU baseline leg at any N (north_star: the 1/2/4/8-GPU figures
    "next to src/crc32c.c timed on the same box's host cores in the same
    run"): rank 0 runs fn() once every rank has finished its GPU timed
    regions and collectives; the other ranks wait for it on the process
    group's store -- a blocking socket read, not a spinning collective, so
    they take no host CPU time from the baseline's threads.  Returns fn()'s
    result on rank 0, None elsewhere."""
    if env.world == 1:
        return fn()
    import datetime

    import torch.distributed as dist

    store = dist.distributed_c10d._get_default_store()
    if env.rank == 0:
        try:
            return fn()
        finally:
            store.set(CPU_BASELINE_KEY, "1")
    store.wait([CPU_BASELINE_KEY], datetime.timedelta(seconds=wait_s))
    return None


def roofline_node(nbytes_per_rank: int, kernel_us_max: float, world: int) -> dict:
    """Node-level roofline fields beside the per-GPU ones: every rank's bytes
    over the slowest rank's kernel time, against N GPUs' HBM peak."""
    achieved = world * nbytes_per_rank / (kernel_us_max * 1e-6) / 1e9 if kernel_us_max > 0 else 0.0
    return {"achieved_node": round(achieved, 1), "peak_node": PEAK_HBM_GBS * world,
            "frac_node": round(achieved / (PEAK_HBM_GBS * world), 4)}


# What every printed line carries (the driver's contract plus this path's
# roofline / cpu_baseline objects); checked by the tests against real lines.
LINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")
ROOFLINE_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "achieved_node", "peak_node", "frac_node")
CPU_BASELINE_KEYS = ("value", "unit", "cores", "kind", "sample")


def line_problems(d: dict, want_cpu: bool = True) -> list:
    """What a bench line lacks against the contract (empty when complete)."""
    bad = ["missing %s" % k for k in LINE_KEYS if k not in d]
    rf = d.get("roofline") or {}
    bad += ["roofline missing %s" % k for k in ROOFLINE_KEYS if k not in rf]
    if "peak_node" in rf and rf["peak_node"] != PEAK_HBM_GBS * d.get("n_gpus", 0):
        bad.append("roofline.peak_node is not n_gpus x %.0f GB/s" % PEAK_HBM_GBS)
    if "frac_node" in rf and not (0 < (rf["frac_node"] or 0) < 1):
        bad.append("roofline.frac_node out of (0, 1)")
    cb = d.get("cpu_baseline")
    if want_cpu:
        if not isinstance(cb, dict):
            bad.append("cpu_baseline is %r" % (cb,))
        else:
            bad += ["cpu_baseline missing %s" % k for k in CPU_BASELINE_KEYS if k not in cb]
            if cb.get("unit") != d.get("unit"):
                bad.append("cpu_baseline unit differs from the line's")
    return bad


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """--gpus N > 1 without a launcher: N ranks under torch.distributed.run,
    started as a child process before this process touches the GPU.  Their
    stdout / stderr are this process's (rank 0's JSON line comes through
    unchanged); the return code is the launcher's."""
    import subprocess

    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if backend == "nccl":
        # (counting devices does not initialise the GPU on this image)
        import torch

        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            print("bench.py: --gpus %d needs %d visible GPUs for one RCCL rank per GPU, found %d "
                  "(BENCH_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs)" % (args.gpus, args.gpus, ndev),
                  file=sys.stderr, flush=True)
            return 2
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


def timed_calls(fn, budget_s: float = 0.25, min_reps: int = 5, max_reps: int = 2000) -> float:
    """Median wall seconds of one call of fn(), over about budget_s of calls."""
    fn()
    t0 = time.perf_counter()
    fn()
    one = max(time.perf_counter() - t0, 1e-7)
    reps = int(min(max_reps, max(min_reps, budget_s / one)))
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def host_block_latency(hdfs, ctx, pk, payload: np.ndarray, want, ref_threads: int, with_ref: bool):
    """The host-resident path at the reference's unit of work (one call over
    one batch that starts and ends in host memory, e.g. one 4 MiB block:
    hadoop_fuse_write_block, src/fuse.c:336-449, one libfuse thread; packets
    cut by hadooprpc.c:815-860): median microseconds per call of
      gpu_pinned / gpu_pageable -- crc32c_batch_host (H2D copy, kernel,
                                   checksums back in host memory),
      product_cpu_1t            -- the product's host path (crc32c_chunks_cpu
                                   per packet on the calling thread),
      reference_1t / _Nt        -- the reference's crc32c.c per chunk as
                                   hadooprpc.c:739 calls it, on 1 thread and
                                   split over N persistent threads (the CPU
                                   baseline leg: oracle/_ref, in-cache),
    each bit-exact against `want` (the reference's checksums)."""
    import torch

    nbytes = int(pk["len"].astype(np.int64).sum())
    nout = hdfs.total_checksums(pk)
    pinned = torch.from_numpy(payload).pin_memory().numpy()
    out = np.zeros(max(nout, 1), np.uint32)
    res = {"bytes": nbytes}
    exact = True
    for name, buf in (("gpu_pinned", pinned), ("gpu_pageable", payload)):
        res[name + "_us"] = round(timed_calls(lambda: ctx.batch_host(buf, pk, out=out)) * 1e6, 2)
        exact = exact and bool(np.array_equal(out[:nout], want))
    res["product_cpu_1t_us"] = round(timed_calls(lambda: hdfs.batch_host_cpu(payload, pk, out=out)) * 1e6, 2)
    exact = exact and bool(np.array_equal(out[:nout], want))
    if with_ref:
        import oracle as oracle_mod

        try:
            ref = oracle_mod.Reference()
            for t in sorted({1, ref_threads}):
                one = ref.block_latency_seconds(payload, pk, out, t, 3)
                reps = int(min(5000, max(5, 0.25 / max(one, 1e-7))))
                res["reference_%dt_us" % t] = round(ref.block_latency_seconds(payload, pk, out, t, reps) * 1e6, 2)
                exact = exact and bool(np.array_equal(out[:nout], want))
        except (FileNotFoundError, OSError):
            pass
    res["bit_exact"] = exact
    return res


# ---- the timed region, shared by the main line and its sub-runs ------------
def settle_for(env, ms: float, fn, collective: bool) -> int:
    """Untimed back-to-back steps for ~ms; returns how many.  Steps that hold
    collective calls run a fixed count (every rank makes the same calls)."""
    import torch

    n = 0
    if ms <= 0:
        return 0
    if collective and env.world > 1:
        for n in range(int(ms * 10)):
            fn(n)
        return n + 1
    # (chunks of 20 launches; the host waits for the chunk before the last
    # one, so the GPU always has one queued and never idles)
    s0 = time.perf_counter()
    prev = None
    while (time.perf_counter() - s0) * 1e3 < ms:
        for _ in range(20):
            fn(n)
            n += 1
        ev = torch.cuda.Event()
        ev.record(env.stream)
        if prev is not None:
            prev.synchronize()
        prev = ev
    return n


def time_steps(env, args, step, warm_step, *, collective=False, use_graph=True, zero=None, probe=None,
               on_abandon=None, settle_ms=None, finish=None, host_lead=True) -> dict:
    """Capture, settle, warm up and time args.steps steps of `step(i, stream)`.

    - The K timed steps are captured into HIP graphs and replayed: each step
      is still one pass of the path over one batch (config 4: the shard
      launch + the RCCL group), but the launches are issued by the GPU's
      command processor instead of one Python -> ctypes -> hipLaunchKernel
      call each (~4.1 us per launch on the host, which bounds one-block
      batches: DESIGN.md section 5).  Capture is agreed over the ranks
      (graphs.capture_agreed): all ranks replay or all issue from the host.
    - The K steps are split in two: the first n_lead of them, then the rest,
      with a timing event between.  The per-launch kernel time is taken over
      the second part only: its launches are queued while the first part's
      run, so it holds neither the host's first issue nor a graph's launch
      latency (~20 us on this stack).  n_lead covers >= 150 us of kernel
      time (at most half the steps).  Both parts are timed steps: the wall
      clock holds all K of them.  A lead of steps of >= 25 us each is issued
      from the host (its first launch starts within a few us, and the main
      part's graph launch hides behind it).  BENCH_CAPTURE_FAIL_RANK=r makes
      rank r's step capture fail (every rank then issues from the host).
    - `finish(stream)` (pipelined steps: config 4's multi plan) runs after
      each part's steps, inside its capture: the part's end event then
      follows every step of it.
    - host_lead=False: the lead is always a graph (config 4, whose warm-up
      steps -- joined one by one -- misprice how far ahead the host issues:
      a host-issued lead of pipelined execs, ~30 us of host time each for
      22 us of GPU time, left the main graph's launch in the kernel window,
      23.4-27.5 against 21.8-22.3 us with a graph lead, round 6).
    - Outputs are zeroed (`zero`) BEFORE the power settle, so the GPU goes
      from settle to warm-up to the timed steps with no idle gap; settle and
      warm-up steps (`warm_step`) write scratch outputs.  Back-to-back
      launches of this kernel push the package to its 1.4 kW cap; the first
      few hundred ride a boost-then-clamp transient 5-12 % slower than the
      steady state.
    Returns the times, max over ranks."""
    import torch
    import torch.distributed as dist

    from hdfs_crc32c_amd.graphs import capture_agreed

    K = args.steps
    world, dev, stream = env.world, env.dev, env.stream
    step_us = host_us = 0.0
    if K > 1:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        h0 = time.perf_counter()
        for i in range(10):
            warm_step(i)
        host_us = (time.perf_counter() - h0) * 1e6 / 10
        e1.record(stream)
        torch.cuda.synchronize()
        step_us = e0.elapsed_time(e1) * 1e3 / 10
    n_lead = 0 if K < 2 else min(K // 2, max(1, -(-150 // max(int(step_us), 1))))
    if world > 1:  # (one split and one lead form on every rank)
        t = torch.tensor([n_lead, step_us, host_us], dtype=torch.float64, device=env.cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        n_lead, step_us, host_us = int(t[0].item()), float(t[1].item()), float(t[2].item())
    parts = [(0, n_lead), (n_lead, K)] if n_lead else [(0, K)]
    # A host-issued lead only where the host runs well ahead of the GPU: a
    # lead issued slower than it executes leaves the GPU idle when the main
    # graph is replayed, and that graph's launch latency lands in the timed
    # part (config 4's multi-plan step, round 5: 25.2 against 24.2 us over a
    # 20-step window).
    lead_host = host_lead and n_lead > 0 and step_us >= 25.0 and host_us < 0.5 * step_us
    graphs, graph_error = {}, None
    if use_graph:
        def capture():
            gs = {}
            try:
                for k, (lo, hi) in enumerate(parts):
                    if lead_host and k == 0:
                        continue
                    g_ = torch.cuda.CUDAGraph()
                    # (thread_local: other threads of the process -- e.g. the process
                    # group's watchdog -- may make HIP calls while this thread captures)
                    with torch.cuda.graph(g_, capture_error_mode="thread_local"):
                        cap = torch.cuda.current_stream(dev)
                        for i in range(lo, hi):
                            step(i, cap.cuda_stream)
                        if finish is not None:  # (pipelined steps join the capture stream before it ends)
                            finish(cap.cuda_stream)
                    gs[k] = g_
                for g_ in gs.values():
                    g_.replay()  # (first replay uploads the graph)
                torch.cuda.synchronize()
            except RuntimeError:
                torch.cuda.synchronize()
                raise
            return gs

        inject = os.environ.get("BENCH_CAPTURE_FAIL_RANK", "") == str(env.rank)
        got, graph_error = capture_agreed(capture, world, env.cdev, probe=probe, on_abandon=on_abandon,
                                          inject_fail=inject)
        graphs = got or {}
        use_graph = bool(got)
    if zero is not None:
        zero()
    torch.cuda.synchronize()
    settle = settle_for(env, args.settle_ms if settle_ms is None else settle_ms, warm_step, collective)
    for i in range(args.warmup):
        warm_step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(parts) + 1)]
    t0 = time.perf_counter()
    evs[0].record(stream)
    for k, (lo, hi) in enumerate(parts):
        if k in graphs:
            graphs[k].replay()
        else:
            for i in range(lo, hi):
                step(i)
            if finish is not None:
                finish(env.sptr)
        evs[k + 1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # avg per step, on the launch stream: over the steps after the lead (all
    # K when there is no lead)
    window_ms = evs[0].elapsed_time(evs[-1]) / max(K, 1)
    lo_t, hi_t = parts[-1]
    kernel_ms = evs[-2].elapsed_time(evs[-1]) / max(hi_t - lo_t, 1)
    own = (elapsed, kernel_ms, window_ms)
    if world > 1:
        t = torch.tensor(own, dtype=torch.float64, device=env.cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms, window_ms = (float(x) for x in t.tolist())
    return {"elapsed": elapsed, "kernel_ms": kernel_ms, "window_ms": window_ms, "parts": parts, "n_lead": n_lead,
            "lead_host": lead_host, "graphs": graphs, "use_graph": use_graph, "graph_error": graph_error,
            "settle": settle, "own_kernel_ms": own[1], "host_issue_us": host_us}


def launch_text(r) -> str:
    if r["use_graph"]:
        return "%s, replayed" % " + ".join(("%d host-issued" if k not in r["graphs"] else "hip graph of %d") % (hi - lo)
                                           for k, (lo, hi) in enumerate(r["parts"]))
    return "host-issued, one launch per step" + (
        "" if r["graph_error"] is None else " (graph capture not agreed: %s)" % r["graph_error"])


def agree_min(env, ok: bool) -> bool:
    from hdfs_crc32c_amd.graphs import agree

    return agree(ok, env.world, env.cdev)


# ---- config 4: the multi-GPU file step (also the default line's sub-object) --
def run_config4(hdfs, args, env) -> dict:
    """Config 4 at this N: a 128 MiB file as 32 x 4 MiB blocks dealt
    round-robin over the ranks (group g of 64 packets on rank g mod N,
    src/fuse.c:580-647 writes a file block by block; hadooprpc.c:815-860
    cuts each block into packets).  One step = crc32c_multi_plan_exec: every
    rank checksums its shard from its own HBM (rank 0 straight into file
    order) and ONE RCCL group lands every peer's block checksums in file
    order on rank 0 (no staging, no copy kernel), captured into the step
    graph.  Buffer b of every rank is its shard of the PCG64 file of seed
    2024 + b, so rank 0 checks the array the LAST timed step gathered
    against the reference over that step's file.  Ranks sharing GPUs over
    gloo (BENCH_DIST_BACKEND=gloo, a rehearsal) run the same shard plans and
    gather with shard.gather_checksums over gloo instead, host-issued."""
    import torch
    import torch.distributed as dist

    from hdfs_crc32c_amd import shard
    from hdfs_crc32c_amd.workloads import synthetic_bytes, uniform_packets

    world, rank, dev = env.world, env.rank, env.dev
    gp = C4_GROUP_PACKETS
    file_pk = uniform_packets(C4_GROUP_PACKETS * C4_BLOCKS)
    file_bytes_total = C4_BLOCKS * shard.BLOCK_BYTES
    lay, shard_sizes = shard.layout(file_pk, gp, world)
    rehearsal = world > 1 and env.backend != "nccl"
    self_send = os.environ.get("BENCH_C4_SELF_SEND") == "1"  # (tests: rank 0's array through RCCL too)
    flags = MULTI_SELF_SEND if self_send else 0
    # CRC32C_MULTI_PIPELINE: step k + 1's shard launch overlaps step k's tail
    # (each step's file and root array its own; joined at the end of every
    # timed part) -- where the step has no gather: with one, the one-GPU
    # model measured the overlapped RCCL group and shard launch slower than
    # stream order (15.4 against 12.8 us graph-replayed).
    # BENCH_C4_PIPELINE=1 / 0 forces it on / off.
    ln0, xs0 = shard.transfers(file_pk, gp, world, flags)
    pipe_env = os.environ.get("BENCH_C4_PIPELINE", "")
    pipeline = not rehearsal and (pipe_env == "1" or (pipe_env != "0" and not int(xs0.shape[0])))
    nbuf = max(1, args.nbuf)
    file0 = synthetic_bytes(file_bytes_total, 2024)
    bufs = []
    for b in range(nbuf):
        fb = file0 if b == 0 else synthetic_bytes(file_bytes_total, 2024 + b)
        bufs.append(torch.from_numpy(shard.rank_payload(fb, lay, shard_sizes, rank)).to(dev))
        del fb
    # this rank's shard plan alone (what the multi plan launches on it): the
    # probe capture with no collective in it, and the shard kernel's time
    mine = shard.plan_packets(file_pk, gp, world, rank, flags)
    ln, xs = shard.transfers(file_pk, gp, world, flags)
    nchk = hdfs.total_checksums(file_pk)
    in_place = rank == 0 and not int(ln[0])
    nlocal = nchk if in_place else int(ln[rank])
    sctx = hdfs.Context(env.local_rank)
    splan = sctx.plan(mine) if mine.size else None
    local_out = torch.zeros(max(nlocal, 1), dtype=torch.int32, device=dev)
    # file b's checksums land in root_outs[b] (rank 0), the warm-up steps' in
    # scratch_roots[b]
    root_outs = [torch.zeros(max(nchk, 1), dtype=torch.int32, device=dev) for _ in range(nbuf)]
    scratch_roots = [torch.zeros_like(root_outs[0]) for _ in range(nbuf)]
    sptr = env.sptr

    state = {}

    def make_multi():
        if world == 1:
            m = hdfs.Multi([env.local_rank])
        else:
            obj = [hdfs.multi_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            m = hdfs.Multi(device=env.local_rank, rank=rank, nranks=world, uid=obj[0])
        state["multi"] = m
        state["mplan"] = m.plan(file_pk, gp, flags | (MULTI_PIPELINE if pipeline else 0))

    def close_multi():
        if state.get("mplan") is not None:
            state["mplan"].close()
        if state.get("multi") is not None:
            state["multi"].close()
        state["mplan"] = state["multi"] = None

    rebuilt = [0]

    def abandon():
        # A rank whose capture failed inside the RCCL group may have left it
        # half-posted: every rank drops its communicator and builds a new one
        # (new id, new crc32c_multi), then issues its steps from the host.
        torch.cuda.synchronize()
        close_multi()
        make_multi()
        rebuilt[0] += 1

    if not rehearsal:
        make_multi()

    def step_into(i, outs_, sp):
        b = i % nbuf
        if rehearsal:
            if splan is not None:
                splan.exec(bufs[b].data_ptr(), local_out.data_ptr(), sp)
            torch.cuda.synchronize()
            got = shard.gather_checksums(local_out.cpu(), file_pk, gp, world, rank, flags)
            if rank == 0:
                outs_[b][:nchk].copy_(torch.from_numpy(got.view(np.int32).copy()))
        else:
            state["mplan"].exec([bufs[b].data_ptr()], outs_[b].data_ptr() if rank == 0 else 0, [sp])

    def step(i, sp=None):
        step_into(i, root_outs, sptr if sp is None else sp)

    def join(sp):
        if not rehearsal:
            state["mplan"].join([sp])

    def warm_step(i):
        step_into(i, scratch_roots, sptr)
        join(sptr)  # (the settle paces itself on the launch stream)

    def probe():
        if splan is None:
            return
        g_ = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g_, capture_error_mode="thread_local"):
                splan.exec(bufs[0].data_ptr(), local_out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
            g_.replay()
        finally:
            torch.cuda.synchronize()

    # correctness gate (outside the timed region): the whole file's checksums
    # gathered on rank 0 against the reference
    step(0)
    join(sptr)
    torch.cuda.synchronize()
    want0 = reference_checksums(file0, file_pk, nchk) if rank == 0 else None
    gate = rank != 0 or bool(np.array_equal(root_outs[0].cpu().numpy().view(np.uint32)[:nchk], want0))

    def zero_roots():
        for o in root_outs:
            o.zero_()

    r = time_steps(env, args, step, warm_step, collective=world > 1, use_graph=not (args.no_graph or rehearsal),
                   zero=zero_roots, probe=probe, on_abandon=abandon, settle_ms=0 if rehearsal else None,
                   finish=join, host_lead=False)
    # every file the timed steps gathered, against the reference (rank 0;
    # root_outs[b] holds the last timed step on buffer b)
    timed = True
    timed_bufs = sorted({i % nbuf for i in range(args.steps)})
    if rank == 0:
        for b in timed_bufs:
            wb = want0 if b == 0 else reference_checksums(synthetic_bytes(file_bytes_total, 2024 + b), file_pk, nchk)
            timed = timed and bool(np.array_equal(root_outs[b].cpu().numpy().view(np.uint32)[:nchk], wb))
    # the shard's plan launch alone (no gather), same buffers, graph-replayed
    # when the step was: what the gather adds to a step is the difference
    # (every rank or none: the timing holds collectives)
    shard_max = None
    rs = None
    if not rehearsal and agree_min(env, splan is not None):
        def sstep(i, sp=None):
            splan.exec(bufs[i % nbuf].data_ptr(), local_out.data_ptr(), sptr if sp is None else sp)
        rs = time_steps(env, args, sstep, sstep, use_graph=r["use_graph"], settle_ms=min(args.settle_ms, 50.0))
        shard_max = rs["kernel_ms"] * 1e3  # (max over ranks)
    # A steady-state window beside the K-step one: 500 graph-replayed steps
    # right after (a 20-step window of 24-us steps holds a few us of window
    # effects: 25.2 against 24.2 us on one box, round 5).
    steady = None
    if not rehearsal and args.steps < 500:
        import copy

        a500 = copy.copy(args)
        a500.steps, a500.warmup = 500, 0
        rst = time_steps(env, a500, step, warm_step, collective=world > 1, use_graph=r["use_graph"],
                         zero=zero_roots, settle_ms=0, finish=join, host_lead=False)
        steady = rst["kernel_ms"] * 1e3
        rst["graphs"].clear()
    exact = agree_min(env, gate and timed)
    launch = launch_text(r)
    # the step graphs hold the RCCL group's captured calls: destroyed before
    # the communicator
    torch.cuda.synchronize()
    r["graphs"].clear()
    if rs is not None:
        rs["graphs"].clear()
    gops = state["mplan"].gather_ops() if state.get("mplan") is not None else None
    close_multi()
    if splan is not None:
        splan.close()
    sctx.close()
    per_rank_max = int(shard_sizes.max()) if len(shard_sizes) else 0
    step_kernel_us = r["kernel_ms"] * 1e3
    return {
        "workload": "128MiB file as 32 x 4MiB blocks round-robin over %d ranks, %s gather of the checksums into "
                    "file order on rank 0 inside every step (config 4)" % (world, "gloo rehearsal" if rehearsal
                                                                           else "RCCL"),
        "n_ranks": world, "steps": args.steps, "warmup": args.warmup,
        "gib_s": round(file_bytes_total * args.steps / r["elapsed"] / GIB, 2),
        "step_us": round(r["elapsed"] / max(args.steps, 1) * 1e6, 3),
        "kernel_step_us": round(step_kernel_us, 3),
        "kernel_step_gib_s": round(file_bytes_total / (step_kernel_us * 1e-6) / GIB, 2),
        # the whole file's bytes per step over the chip's HBM peak x ranks
        "frac_of_hbm_roofline": round(file_bytes_total / (step_kernel_us * 1e-6) / 1e9 / (PEAK_HBM_GBS * world), 4),
        "shard_kernel_us": None if shard_max is None else round(shard_max, 3),
        "shard_bytes_max": per_rank_max,
        "shard_frac_of_hbm_roofline": None if not shard_max else
        round(per_rank_max / (shard_max * 1e-6) / 1e9 / PEAK_HBM_GBS, 4),
        # (what the in-step gather adds: the step minus the shard's launch;
        # none without transfers -- N = 1 in place)
        "gather_us": None if (shard_max is None or not int(xs.shape[0])) else round(step_kernel_us - shard_max, 3),
        "transfers": int(xs.shape[0]), "self_send": self_send,
        # (RCCL operations per step, whole communicator; packed: one send per
        # rank into rank 0's staging array + the scatter kernel)
        "gather_ops": None if gops is None else gops[0], "gather_packed": None if gops is None else gops[1],
        "bit_exact": exact,
        "bit_exact_checks": {"before_warmup_file0": gate,
                             "timed_files_buf%s" % "_".join(str(b) for b in timed_bufs): timed} if rank == 0 else None,
        "pipelined": pipeline,
        "launch": launch, "lead_steps": "host-issued" if (r["lead_host"] or not r["use_graph"]) else "graph",
        "host_issue_us_per_step": round(r["host_issue_us"], 2),
        "kernel_step_us_500": None if steady is None else round(steady, 3),
        "frac_of_hbm_roofline_500": None if steady is None else
        round(file_bytes_total / (steady * 1e-6) / 1e9 / (PEAK_HBM_GBS * world), 4),
        "communicator_rebuilt": rebuilt[0], "settle_launches": r["settle"],
        "mode": "gloo rehearsal (ranks share GPUs; not a measurement)" if rehearsal else "rccl",
    }


def run_strong(hdfs, args, env, ctx) -> dict:
    """The one config-2 batch (4096 x 64 KiB packets, 256 MiB) split over the
    ranks (strong scaling): rank r checksums packets
    [r N/W, (r+1) N/W) from its own HBM, no data-path collective; value =
    256 MiB per step / the slowest rank's time."""
    import torch

    from hdfs_crc32c_amd.workloads import synthetic_bytes, uniform_packets

    world, rank, dev = env.world, env.rank, env.dev
    full = uniform_packets(4096)
    lo, hi = rank * full.size // world, (rank + 1) * full.size // world
    pk = full[lo:hi].copy()
    pk["payload_off"] -= pk["payload_off"][0]
    pk["out_idx"] -= pk["out_idx"][0]
    nbytes = int(pk["len"].astype(np.int64).sum())
    total_bytes = int(full["len"].astype(np.int64).sum())
    nout = hdfs.total_checksums(pk)
    plan = ctx.plan(pk)
    nbuf = max(1, args.nbuf)
    payload0 = synthetic_bytes(nbytes, 3030 + rank)
    bufs = [torch.from_numpy(payload0).to(dev)]
    g = torch.Generator(device=dev)
    g.manual_seed(4321 + rank)
    for _ in range(1, nbuf):
        bufs.append(torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev, generator=g))
    outs = [torch.zeros(max(nout, 1), dtype=torch.int32, device=dev) for _ in range(nbuf)]
    scratch = [torch.zeros_like(o) for o in outs]
    sptr = env.sptr

    def step(i, sp=None):
        plan.exec(bufs[i % nbuf].data_ptr(), outs[i % nbuf].data_ptr(), sptr if sp is None else sp)

    def warm(i):
        plan.exec(bufs[i % nbuf].data_ptr(), scratch[i % nbuf].data_ptr(), sptr)

    def zero():
        for o in outs:
            o.zero_()

    r = time_steps(env, args, step, warm, use_graph=not args.no_graph, zero=zero)
    want = reference_checksums(payload0, pk, nout)
    exact = args.steps < nbuf or bool(np.array_equal(outs[0].cpu().numpy().view(np.uint32)[:nout], want))
    exact = agree_min(env, exact)
    plan.close()
    kernel_us = r["kernel_ms"] * 1e3
    return {
        "workload": "the config-2 batch (4096 x 64KiB packets, 256 MiB) split over %d ranks" % world,
        "n_ranks": world, "packets_per_rank": int(pk.size), "steps": args.steps,
        "gib_s": round(total_bytes * args.steps / r["elapsed"] / GIB, 2),
        "step_us": round(r["elapsed"] / max(args.steps, 1) * 1e6, 3),
        "kernel_us_max_rank": round(kernel_us, 3),
        "frac_of_hbm_roofline_per_gpu": round(nbytes / (kernel_us * 1e-6) / 1e9 / PEAK_HBM_GBS, 4),
        "bit_exact": exact, "launch": launch_text(r), "settle_launches": r["settle"],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # Defaults measure the steady state: the first ~500 back-to-back launches
    # ride a power-management transient (boost, then an overshooting clamp at
    # the 1.4 kW package cap).  2500 launches take ~0.1 s.
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--config", default="c2", type=config_name,
                    help="c2 | c3 | c4 | c5 | c2b1536 | c2b1000 | c2b<bpc> | c2u | c2t | c3u")
    ap.add_argument("--nbuf", type=int, default=4, help="rotating payload buffers (defeat the 256 MiB L3)")
    ap.add_argument("--cpu-seconds", type=float, default=4.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host", action="store_true")
    ap.add_argument("--no-config4", action="store_true", help="skip the config4 sub-object of the c2 line")
    ap.add_argument("--no-strong", action="store_true", help="skip the strong_scaling sub-object of the c2 line")
    ap.add_argument("--sub-timeout-s", type=float, default=420.0,
                    help="bound on the config4 + strong_scaling sub-runs, the CPU baseline and the teardown after "
                         "them: past it rank 0 prints the main line with the sub-objects marked timed out and every "
                         "rank exits")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak (default): every rank checksums its own config batch; strong: the config-2/5 batch's "
                         "packets are split evenly over the ranks (SURVEY.md section 8e)")
    ap.add_argument("--no-graph", action="store_true",
                    help="issue the timed launches one by one from Python instead of replaying them from a graph")
    ap.add_argument("--two-streams", action="store_true",
                    help="also time 1000 batches alternated over two streams (their launches overlap, so a "
                         "rocprofv3 run of the bench would average overlapped durations: off by default)")
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="untimed back-to-back steps before the warm-up, past the power transient (0: none)")
    ap.add_argument("--host-sweep", action="store_true",
                    help="also time the host-resident path per call against the host CPU over batch sizes from "
                         "one 64 KiB packet to 256 MiB (N = 1; adds host_sweep to the line)")
    ap.add_argument("--host-multi-devices", type=int, default=1,
                    help="GPUs crc32c_multi_batch_host deals the host-resident batch over at N = 1 (0: skip)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d: the launcher and the flag disagree"
              % (os.environ["WORLD_SIZE"], args.gpus), file=sys.stderr, flush=True)
        sys.exit(2)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # One process per GPU over RCCL (the "nccl" backend).  BENCH_DIST_BACKEND=gloo
    # rehearses the N > 1 path with ranks sharing the visible GPUs (their
    # collectives then go through host memory); never used for a measurement.
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend != "nccl":
        local_rank = local_rank % max(1, ndev)
    elif local_rank >= ndev:
        print("bench.py: rank %d (local rank %d) has no GPU of its own: %d visible; one RCCL rank per GPU"
              % (rank, local_rank, ndev), file=sys.stderr, flush=True)
        sys.exit(2)
    torch.cuda.set_device(local_rank)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)

    hdfs = load_package()
    hdfs.lib()

    from hdfs_crc32c_amd import shard
    from hdfs_crc32c_amd.workloads import config_packets, synthetic_bytes

    dev = torch.device("cuda", local_rank)
    stream = torch.cuda.current_stream(dev)
    env = SimpleNamespace(world=world, rank=rank, local_rank=local_rank, backend=backend, dev=dev, stream=stream,
                          sptr=stream.cuda_stream,
                          cdev=dev if backend == "nccl" else torch.device("cpu"))  # where collectives run
    cdev = env.cdev

    if args.config == "c4":  # config 4 as the main line (builder's runs): its sub-run, reported flat
        c4 = run_config4(hdfs, args, env)
        if rank == 0:
            kus = c4["kernel_step_us"]
            line = {
                "metric": baseline_metric(), "value": c4["gib_s"], "unit": "GiB/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(c4["step_us"] * 1e-3, 5),
                "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u32",
                "data": "synthetic (PCG64 file bytes, %d rotating files)" % max(1, args.nbuf),
                "config": {"workload": c4["workload"], "config": "c4",
                           "parallelism": "dp%d (block shards, crc32c_multi_plan: RCCL send/recv gather of the "
                                          "checksums to rank 0 inside every step)" % world},
                # (the step's bytes are the whole file's, over N GPUs: peak and
                # frac are node-level here; the _node fields say the same)
                "roofline": dict({"bound": "hbm", "achieved": round(C4_BLOCKS * shard.BLOCK_BYTES / (kus * 1e-6) / 1e9, 1),
                                  "peak": PEAK_HBM_GBS * world, "unit": "GB/s", "frac": c4["frac_of_hbm_roofline"],
                                  "traffic": None, "kernel": KERNEL_NAME, "kernel_avg_us": kus,
                                  "algorithmic_bytes_per_launch": C4_BLOCKS * shard.BLOCK_BYTES,
                                  "shard_frac_per_gpu": c4["shard_frac_of_hbm_roofline"]},
                                 **roofline_node(C4_BLOCKS * shard.BLOCK_BYTES // world, kus, world)),
                "cpu_baseline": None, "bit_exact_vs_reference": c4["bit_exact"], "config4": c4,
            }
        if not args.no_cpu:  # (rank 0, after every rank's GPU work; the others wait)
            from hdfs_crc32c_amd.workloads import uniform_packets

            cb = cpu_baseline_on_rank0(env, lambda: cpu_baseline(
                uniform_packets(C4_GROUP_PACKETS * C4_BLOCKS), synthetic_bytes(C4_BLOCKS * shard.BLOCK_BYTES, 2024),
                args.cpu_seconds))
            if rank == 0:
                line["cpu_baseline"] = cb
        if rank == 0:
            print(json.dumps(line), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    pk, workload = config_packets(args.config)
    if args.scaling == "strong" and world > 1:
        if args.config not in ("c2", "c5") or pk.size % world:
            raise SystemExit("--scaling strong needs config c2/c5 and a rank count dividing %d" % pk.size)
        per = pk.size // world
        pk = pk[rank * per:(rank + 1) * per].copy()  # this rank's packets, rebased
        pk["payload_off"] -= pk["payload_off"][0]
        pk["out_idx"] -= pk["out_idx"][0]
        workload += ", strong scaling: packets split over %d ranks" % world
    nbuf = args.nbuf if args.config not in ("c3", "c3u") else 1
    nbytes = int(pk["len"].astype(np.int64).sum())
    extent = int((pk["payload_off"] + pk["len"]).max())
    nout = hdfs.total_checksums(pk)

    ctx = hdfs.Context(local_rank)
    plan = ctx.plan(pk)
    # buffer 0: PCG64 host bytes (checked against the CPU path below); the
    # rest: device-generated random bytes
    payload0 = synthetic_bytes(extent, 2024 + rank)
    bufs = [torch.from_numpy(payload0).to(dev)]
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    for b in range(1, nbuf):
        bufs.append(torch.randint(0, 256, (extent,), dtype=torch.uint8, device=dev, generator=g))
    outs = [torch.zeros(max(nout, 1), dtype=torch.int32, device=dev) for _ in range(nbuf)]
    sptr = env.sptr

    def step(i, sp=None):
        b = i % nbuf
        plan.exec(bufs[b].data_ptr(), outs[b].data_ptr(), sptr if sp is None else sp)

    # correctness gate (outside the timed region): every buffer-0 checksum
    step(0)
    torch.cuda.synchronize()
    want = reference_checksums(payload0, pk, nout)
    got0 = outs[0].cpu().numpy().view(np.uint32)[:nout]
    bit_exact = bool(np.array_equal(got0, want))
    gate_exact = bit_exact

    # settle and warm-up steps write a scratch copy of the outputs (same
    # payloads, same plan), so the checks after the timed region see only
    # what the timed launches wrote
    scratch_outs = [torch.zeros_like(o) for o in outs]

    def warm_step(i):
        b = i % nbuf
        plan.exec(bufs[b].data_ptr(), scratch_outs[b].data_ptr(), sptr)

    def zero_outs():
        for o in outs:
            o.zero_()

    r = time_steps(env, args, step, warm_step, use_graph=not args.no_graph, zero=zero_outs)
    elapsed, kernel_ms, window_ms = r["elapsed"], r["kernel_ms"], r["window_ms"]
    use_graph, graphs, parts = r["use_graph"], r["graphs"], r["parts"]

    # Correctness of the timed launches themselves (outside the timed region):
    # the checksums the last timed launch on buffer 0 (PCG64 host bytes) and
    # on buffer 1 (device random bytes, copied back) wrote, against the
    # reference's crc32c.c.
    timed_checks = {}
    if args.steps > 0:
        timed_checks["timed_buf0"] = bool(np.array_equal(outs[0].cpu().numpy().view(np.uint32)[:nout], want))
        if nbuf > 1 and args.steps > 1:
            w1 = reference_checksums(bufs[1].cpu().numpy(), pk, nout)
            timed_checks["timed_buf1_device_random"] = bool(
                np.array_equal(outs[1].cpu().numpy().view(np.uint32)[:nout], w1))
    timed_exact = all(timed_checks.values())
    eager_ms = None
    if use_graph:  # the same steps issued one by one from the host, for comparison
        # (after the checks above the GPU sat idle for a while: settle again,
        # or the host-issued launches ride the power transient)
        settle_for(env, args.settle_ms, warm_step, False)
        ne = min(args.steps, 500)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(ne):
            step(i)
        e1.record(stream)
        torch.cuda.synchronize()
        eager_ms = e0.elapsed_time(e1) / ne

    if world > 1:
        ok = torch.tensor([1 if bit_exact and timed_exact else 0], dtype=torch.int32, device=cdev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        bit_exact = bool(ok.item())
    # Configs 2/5 (weak scaling, independent batches): RCCL gather of every
    # rank's checksum array to rank 0 after the timed region, timed on its
    # own.  (Config 4's gather is inside every step: the config4 sub-object.)
    gather_ms = None
    if world > 1:
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        send = outs[0].to(cdev)
        gathered = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
        dist.gather(send, gathered, dst=0)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3

    total_bytes = nbytes * world * args.steps
    value = total_bytes / elapsed / GIB
    achieved_gbs = nbytes / (kernel_ms * 1e-3) / 1e9

    # Read-side verification (crc32c_plan_verify) of the rotating buffers
    # against their checksums (outs[b] now holds buffer b's), timed the same
    # way (rank 0, reported beside the main line).
    verify = None
    if rank == 0:
        res = torch.zeros(2, dtype=torch.int32, device=dev)
        for i in range(200):
            plan.verify(bufs[i % nbuf].data_ptr(), outs[i % nbuf].data_ptr(), res.data_ptr(), sptr)
        # 1000 launches (~45 ms at config 2): a window of 200 fell inside the
        # power controller's post-idle clamp on some boxes
        nv = 1000
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(nv):
            plan.verify(bufs[i % nbuf].data_ptr(), outs[i % nbuf].data_ptr(), res.data_ptr(), sptr)
        e1.record(stream)
        torch.cuda.synchronize()
        rr = res.cpu().numpy().view(np.uint32)
        verify = {"gib_s": round(nbytes * nv / (e0.elapsed_time(e1) * 1e-3) / GIB, 1),
                  "kernel_avg_us": round(e0.elapsed_time(e1) / nv * 1e3, 2),
                  "mismatches": int(rr[0]), "clean": bool(rr[0] == 0 and rr[1] == 0xFFFFFFFF),
                  "launch": "host-issued"}
        vgraph = None
        if use_graph:  # also replayed from a graph like the timed exec steps
            # A plan orders its verify launches across streams with an event
            # wait when the stream changes; one launch on the capture stream
            # first keeps that wait out of the capture.
            cs = torch.cuda.Stream(device=dev)
            torch.cuda.synchronize()
            plan.verify(bufs[0].data_ptr(), outs[0].data_ptr(), res.data_ptr(), cs)
            torch.cuda.synchronize()
            try:
                vgraph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(vgraph, stream=cs, capture_error_mode="thread_local"):
                    for i in range(nv):
                        plan.verify(bufs[i % nbuf].data_ptr(), outs[i % nbuf].data_ptr(), res.data_ptr(), cs)
                vgraph.replay()
            except RuntimeError:
                vgraph = None
            torch.cuda.synchronize()
        if vgraph is not None:
            e0.record(stream)
            vgraph.replay()
            e1.record(stream)
            torch.cuda.synchronize()
            rr = res.cpu().numpy().view(np.uint32)
            verify["graph_kernel_avg_us"] = round(e0.elapsed_time(e1) / nv * 1e3, 2)
            verify["graph_clean"] = bool(rr[0] == 0 and rr[1] == 0xFFFFFFFF)
            verify["clean"] = verify["clean"] and verify["graph_clean"]
            # The same nv-launch graph form for exec, right after (into the
            # scratch outputs): what the verify graph is read against, and a
            # steady-state exec figure beside the timed window's.
            try:
                plan.exec(bufs[0].data_ptr(), scratch_outs[0].data_ptr(), cs)
                torch.cuda.synchronize()
                egraph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(egraph, stream=cs, capture_error_mode="thread_local"):
                    for i in range(nv):
                        plan.exec(bufs[i % nbuf].data_ptr(), scratch_outs[i % nbuf].data_ptr(), cs)
                egraph.replay()
                torch.cuda.synchronize()
                e0.record(stream)
                egraph.replay()
                e1.record(stream)
                torch.cuda.synchronize()
                verify["exec_graph_kernel_avg_us"] = round(e0.elapsed_time(e1) / nv * 1e3, 2)
            except RuntimeError:
                torch.cuda.synchronize()

    # The box's own streaming-read rate over the same rotating buffers, right
    # after the timed region (same power state): a plain grid-stride read
    # with non-temporal loads (stream_probe.hip shape 2, 512 x 256 threads,
    # the best plain shape of tools/probe_sweep.py), timed like a step.  It
    # prices the kernel against what this chip actually streams, beside the
    # 8 TB/s datasheet peak.  Rank 0, N = 1 only.
    read_probe = None
    if rank == 0 and world == 1 and nbuf > 1:
        probe_out = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
        L = hdfs.debug_lib()  # the read probe lives in the debug library, not the product

        def probe(i):
            rc = L.crc32c_debug_stream_probe(bufs[i % nbuf].data_ptr(), extent, probe_out.data_ptr(), 512, 2, sptr)
            if rc:
                raise RuntimeError("stream probe rc %d" % rc)

        for i in range(50):
            probe(i)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        np_ = 500
        for i in range(np_):
            probe(i)
        e1.record(stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / np_ * 1e3
        probe_gbs = extent / (us * 1e-6) / 1e9
        read_probe = {"us_per_pass": round(us, 2), "GB_s": round(probe_gbs, 1),
                      "kernel_frac_of_probe": round(achieved_gbs / probe_gbs, 4),
                      "shape": "grid-stride 16 B nt loads, 4 in flight per lane, 512 x 256 threads"}

    # Independent batches on two streams (opt-in, rank 0, beside the main
    # line, which stays one stream so that one step = one launch): the next
    # launch's workgroups start on the CUs the previous one has released.
    two_streams = None
    if args.two_streams and rank == 0 and world == 1 and nbuf > 1:
        ss = [torch.cuda.Stream(device=dev) for _ in range(2)]

        def two(n):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for s in ss:
                s.wait_event(e0)
            for i in range(n):
                plan.exec(bufs[i % nbuf].data_ptr(), outs[i % nbuf].data_ptr(), ss[i % 2])
            for s in ss:
                ej = torch.cuda.Event()
                ej.record(s)
                stream.wait_event(ej)
            e1.record(stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e-3

        two(200)
        n2 = 1000
        dt = two(n2)
        two_streams = {"gib_s": round(nbytes * n2 / dt / GIB, 1), "us_per_batch": round(dt / n2 * 1e6, 2),
                       "batches": n2}

    # Host-resident rate (crc32c_batch_host: pinned host batch -> GPU ->
    # checksums in host memory), every rank at once on its own GPU and PCIe
    # link; the node-level rate is all ranks' bytes / the slowest rank's time.
    # Beside it, the link's ceiling: a plain pinned H2D copy of the same bytes.
    host = h2d = host_multi = host_latency = host_sweep = None
    if not args.no_host:
        pinned = torch.from_numpy(payload0).pin_memory()
        hp = pinned.numpy()
        hout = np.zeros(max(nout, 1), np.uint32)  # caller-owned output, as hadooprpc.c's packet buffer
        ctx.batch_host(hp, pk, out=hout)  # warm (allocates staging)
        reps = 5

        def slowest(dt):
            if world > 1:
                t = torch.tensor([dt], dtype=torch.float64, device=cdev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                dt = float(t[0])
            return dt

        if world > 1:
            dist.barrier()
        h0 = time.perf_counter()
        for _ in range(reps):
            ctx.batch_host(hp, pk, out=hout)
        host = round(world * nbytes * reps / slowest(time.perf_counter() - h0) / GIB, 2)
        timed_checks["host_resident"] = bool(np.array_equal(hout[:nout], want))
        if not timed_checks["host_resident"]:
            bit_exact = False
        dst = torch.empty(pinned.numel(), dtype=torch.uint8, device=dev)
        dst.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        h0 = time.perf_counter()
        for _ in range(reps):
            dst.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
        h2d = round(world * pinned.numel() * reps / slowest(time.perf_counter() - h0) / GIB, 2)
        del dst
        # The N-link lever: crc32c_multi_batch_host deals the batch's 4 MiB
        # blocks over --host-multi-devices GPUs from one process, each over
        # its own PCIe link (default 1: an N = 1 line uses one GPU even on a
        # node that shows eight; at N > 1 every rank's own link is measured
        # above instead).
        if world == 1 and args.host_multi_devices > 0:
            ndv = min(args.host_multi_devices, torch.cuda.device_count())
            devs = [(local_rank + k) % torch.cuda.device_count() for k in range(ndv)]
            m = hdfs.Multi(devs)
            try:
                mout = m.batch_host(hp, pk, group_packets=64)
                exact_multi = bool(np.array_equal(mout[:nout], want))
                h0 = time.perf_counter()
                for _ in range(reps):
                    m.batch_host(hp, pk, group_packets=64)
                host_multi = {"gib_s": round(nbytes * reps / (time.perf_counter() - h0) / GIB, 2),
                              "devices": ndv, "bit_exact": exact_multi, "entry": "crc32c_multi_batch_host"}
                timed_checks["host_resident_multi"] = exact_multi
                bit_exact = bit_exact and exact_multi
            finally:
                m.close()
        # Per call, at this config's batch (config 3: the reference's unit,
        # one 4 MiB block), against the host CPU; --host-sweep: over sizes.
        if world == 1:
            quota = cpu_quota()[1]
            qthreads = max(1, min(os.cpu_count() or 1, int(math.ceil(quota)) if quota else 16))
            host_latency = host_block_latency(hdfs, ctx, pk, payload0, want, qthreads, not args.no_cpu)
            timed_checks["host_latency"] = host_latency["bit_exact"]
            if args.host_sweep:
                from hdfs_crc32c_amd.workloads import uniform_packets

                host_sweep = []
                for npk in (1, 4, 16, 64, 256, 1024, 4096):
                    spk = uniform_packets(npk)
                    sp = synthetic_bytes(npk * 65536, 77 + npk)
                    sw = reference_checksums(sp, spk, hdfs.total_checksums(spk))
                    rr = host_block_latency(hdfs, ctx, spk, sp, sw, qthreads, not args.no_cpu)
                    host_sweep.append(rr)
                    timed_checks["host_sweep_%d" % npk] = rr["bit_exact"]
                cross = [x["bytes"] for x in host_sweep
                         if "reference_1t_us" in x and x["gpu_pinned_us"] < x["reference_1t_us"]]
                host_sweep = {"sizes": host_sweep,
                              "gpu_pinned_beats_reference_1t_from_bytes": min(cross) if cross else None}

    line = None
    if rank == 0:
        pmc = latest_pmc(os.path.join(ROOT, "profiles"), args.config)
        traffic = traffic_commit = None
        if (pmc and pmc.get("config") == args.config
                and PRODUCTION_KERNEL in pmc.get("dispatch_meta", {}).get("Kernel_Name", "")):
            traffic = pmc.get("hbm_bytes_per_launch")
            traffic_commit = pmc.get("commit")
        line = {
            "metric": baseline_metric(),
            "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "settle_launches": r["settle"],
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True, "scaling": "strong" if (args.scaling == "strong" and world > 1) else "weak",
            "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (PCG64 host bytes + device random bytes, %d rotating %d MiB buffers per rank)"
                    % (nbuf, extent >> 20),
            "config": {"workload": workload, "config": args.config, "packets_per_rank": int(pk.size),
                       "packet_bytes": int(pk["len"][0]), "bytes_per_checksum": sorted(set(int(x) for x in pk["bpc"])),
                       "payload_bytes_per_rank": nbytes, "checksums_per_rank": nout,
                       "parallelism": "dp%d (independent shards, %s gather of checksums after timing)"
                                      % (world, "RCCL" if backend == "nccl" else backend + " rehearsal")},
            "roofline": dict({"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / PEAK_HBM_GBS, 4), "traffic": traffic,
                         "traffic_source": None if traffic is None else
                         "rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE per launch, profiles/ summary at commit %s"
                         % traffic_commit,
                         "kernel": KERNEL_NAME, "kernel_avg_us": round(kernel_ms * 1e3, 2),
                         "kernel_timing": "HIP events on the launch stream around timed steps %d..%d (the first %d "
                                          "timed steps, launched first, cover the %s latency); max over ranks"
                                          % (parts[-1][0] + 1, parts[-1][1], r["n_lead"],
                                             "graph launch" if use_graph else "first host issue"),
                         "lead_steps": "host-issued" if (r["lead_host"] or not use_graph) else "graph",
                         "host_issue_us_per_step": round(r["host_issue_us"], 2),
                         "window_avg_us_all_steps": round(window_ms * 1e3, 2),
                         "algorithmic_bytes_per_launch": nbytes}, **roofline_node(nbytes, kernel_ms * 1e3, world)),
            "cpu_baseline": None,  # (filled in last: after every GPU timed region, below)
            "bit_exact_vs_reference": bit_exact and timed_exact,
            "bit_exact_checks": dict({"before_warmup_buf0": gate_exact}, **timed_checks),
            "host_resident_gib_s": host,
            "host_h2d_copy_gib_s": h2d,
            "host_resident_ranks": world if host is not None else None,
            "host_resident_multi": host_multi,
            "host_resident_per_call": host_latency,
            "host_sweep": host_sweep,
            "verify": verify,
            "two_streams": two_streams,
            "box_read_probe": read_probe,
            "gather_ms": None if gather_ms is None else round(gather_ms, 3),
            "launch": launch_text(r),
            "eager_ms_per_step": None if eager_ms is None else round(eager_ms, 5),
            "config4": None,
            "strong_scaling": None,
        }

    # The other two shapes of the 1/2/4/8-GPU curve, on the default line at
    # every N (the driver only runs the default command): config 4's file
    # step with its in-step RCCL gather, and config 2 split over the ranks.
    # They run after the main line is complete, under a watchdog: a sub-run
    # that raises is reported in its sub-object, and one that hangs (a
    # collective some rank never joins) or a teardown that does cannot cost
    # the main line.
    sub = args.config == "c2" and args.scaling == "weak" and not (args.no_config4 and args.no_strong)
    wd = SubRunWatchdog(args.sub_timeout_s, line) if sub else None
    if sub:
        wd.start()
        if not args.no_config4:
            line_set(line, "config4", wd.run("config4", run_config4, hdfs, args, env))
        if not args.no_strong and not wd.failed:
            line_set(line, "strong_scaling", wd.run("strong_scaling", run_strong, hdfs, args, env, ctx))
    # The CPU baseline, last: rank 0's host cores once no rank has GPU work or
    # collectives left (at N > 1 the other ranks wait on the store), so it
    # neither competes with the timed regions nor holds peers in a collective.
    if not args.no_cpu:
        line_set(line, "cpu_baseline", cpu_baseline_on_rank0(env, lambda: cpu_baseline(pk, payload0,
                                                                                      args.cpu_seconds)))
    if wd is not None:
        wd.publish()
    elif line is not None:
        print(json.dumps(line), flush=True)
    plan.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    if wd is not None:
        wd.cancel()


def line_set(line, key, value):
    if line is not None:
        line[key] = value


class SubRunWatchdog:
    """Bounds the sub-runs that follow the main measurement (and the teardown
    after them).  A sub-run that raises is recorded as {"error": ...} in its
    sub-object and the sub-runs after it are skipped (a rank that left a
    collective sequence would leave its peers waiting).  If the bound passes
    first, rank 0 prints the main line -- the sub-objects it has, the others
    marked timed out -- and every rank ends its process: the peers of a hung
    collective are stuck in the same place, each under its own watchdog."""

    def __init__(self, seconds, line):
        import threading

        self.seconds, self.line = seconds, line
        self.failed = False
        self.printed = False
        self.current = None
        self.lock = threading.Lock()
        self.timer = threading.Timer(seconds, self._fire)
        self.timer.daemon = True

    def start(self):
        self.timer.start()

    def run(self, name, fn, *a):
        self.current = name
        try:
            return fn(*a)
        except Exception as e:  # (reported, not raised: the main line is already measured)
            self.failed = True
            return {"error": "%s: %s" % (type(e).__name__, e)}
        finally:
            self.current = None

    def publish(self):
        with self.lock:
            if self.line is not None and not self.printed:
                print(json.dumps(self.line), flush=True)
                self.printed = True

    def cancel(self):
        self.timer.cancel()

    def _fire(self):
        with self.lock:
            if self.line is not None and not self.printed:
                for key in ("config4", "strong_scaling"):
                    if self.line.get(key) is None:
                        self.line[key] = {"error": "timed out: the sub-runs passed --sub-timeout-s %.0f s%s"
                                          % (self.seconds, " in " + self.current if self.current else "")}
                print(json.dumps(self.line), flush=True)
                self.printed = True
            sys.stdout.flush()
            sys.stderr.write("bench: sub-run watchdog fired after %.0f s; exiting\n" % self.seconds)
            sys.stderr.flush()
            os._exit(0)


if __name__ == "__main__":
    main()
