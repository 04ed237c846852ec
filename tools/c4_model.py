#!/usr/bin/env python3
"""Measured parts of a model of config 4 at N = 8.

At N = 8 every rank checksums 4 of the 32 blocks (a 16 MiB shard: 256
packets of 64 KiB) and ranks 1-7 each send 4 x 8192 checksums (128 KiB) to
rank 0, which scatters them into file order.  On a one-GPU box this times,
per step (HIP events on the launch stream, 1000 steps after 200 warm-up):

  shard_graph / shard_eager -- the production kernel over one rank's 16 MiB
                               shard, graph-replayed / host-issued;
  multi_in_place            -- crc32c_multi_plan_exec over the same shard on
                               a 1-rank communicator (rank 0 writes in place:
                               no RCCL call);
  multi_self_send           -- the same with CRC32C_MULTI_SELF_SEND: the
                               shard's 128 KiB go through one RCCL send/recv
                               group to rank 0's own staging slot, then the
                               scatter kernel -- a lower bound for one peer's
                               gather at N = 8;
  multi_self_send_4x        -- the same with the shard's four groups placed
                               apart in the output (four 32 KiB ranges, as
                               one peer's at N = 8, where its 4 blocks are 8
                               blocks apart in file order): packed (one
                               send/recv pair into the staging array, then
                               the scatter kernel) and _per_group (four
                               pairs, CRC32C_MULTI_PER_GROUP_RECV).

Each multi step is also captured (kernel + RCCL group) into a graph of 100
steps and replayed (*_graph_us), as bench.py replays config 4's steps.

  pipe_in_place / pipe_self_send -- the same two with CRC32C_MULTI_PIPELINE
                               (consecutive steps into 4 rotating root arrays
                               overlap; joined at the end), host-issued and
                               graph-replayed, checked against the plain
                               plan's checksums.

Prints one JSON line.  The model: step(N = 8) ~= shard time + gather time,
with the gather at least (multi_self_send - multi_in_place); graph-replayed,
step(N = 8) ~= multi_self_send_graph (the shard plus one RCCL group)."""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench

    hdfs = bench.load_package()
    hdfs.lib()
    from hdfs_crc32c_amd.workloads import synthetic_bytes, uniform_packets

    dev = torch.device("cuda", 0)
    pk = uniform_packets(256)  # one rank's shard at N = 8: 4 blocks x 64 packets
    nbytes = 256 * 65536
    payload = torch.from_numpy(synthetic_bytes(nbytes + 16, 5)).to(dev)
    out = torch.zeros(256 * 128, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def timed(fn, n=1000, warm=200):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(n):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n * 1e3  # us per call

    res = {"shard_bytes": nbytes, "shard_packets": 256}
    ctx = hdfs.Context(0)
    plan = ctx.plan(pk)
    res["shard_eager_us"] = round(timed(lambda: plan.exec(payload.data_ptr(), out.data_ptr(), stream.cuda_stream)), 3)
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(device=dev)  # (capture stream)
    plan.exec(payload.data_ptr(), out.data_ptr(), cs.cuda_stream)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=cs, capture_error_mode="thread_local"):
        for _ in range(100):
            plan.exec(payload.data_ptr(), out.data_ptr(), cs.cuda_stream)
    g.replay()
    torch.cuda.synchronize()
    res["shard_graph_us"] = round(timed(lambda: g.replay(), n=50, warm=5) / 100, 3)
    plan.close()
    # (multi_self_send_4x: the four groups' checksum ranges 37 apart in the
    # output, so they do not merge -- four 32 KiB transfers, one N = 8 peer's
    # pattern: its 4 blocks are 8 blocks apart in file order)
    pk4 = pk.copy()
    gap = 37
    pk4["out_idx"] = np.array([(i // 64) * (64 * 128 + gap) + (i % 64) * 128 for i in range(pk.size)], np.uint64)
    out4 = torch.zeros(4 * (64 * 128 + gap), dtype=torch.int32, device=dev)
    for name, flags, pkm, o in (("multi_in_place", 0, pk, out),
                                ("multi_self_send", hdfs.CRC32C_MULTI_SELF_SEND, pk, out),
                                ("multi_self_send_4x", hdfs.CRC32C_MULTI_SELF_SEND, pk4, out4),
                                ("multi_self_send_4x_per_group",
                                 hdfs.CRC32C_MULTI_SELF_SEND | hdfs.CRC32C_MULTI_PER_GROUP_RECV, pk4, out4)):
        m = hdfs.Multi([0])
        mp = m.plan(pkm, 64, flags)
        if "_4x" in name:
            res[name + "_gather_ops"] = list(mp.gather_ops())
        res[name + "_us"] = round(timed(lambda: mp.exec([payload.data_ptr()], o.data_ptr(), [stream.cuda_stream])), 3)
        if "_4x" in name:
            got = o.cpu().numpy().reshape(4, -1)[:, :64 * 128].reshape(-1)
            res[name + "_exact"] = bool(np.array_equal(got, out.cpu().numpy()))
        # the whole step (kernel + RCCL group) captured 100 times into one graph
        mp.exec([payload.data_ptr()], o.data_ptr(), [cs.cuda_stream])
        torch.cuda.synchronize()
        try:
            gm = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gm, stream=cs, capture_error_mode="thread_local"):
                for _ in range(100):
                    mp.exec([payload.data_ptr()], o.data_ptr(), [cs.cuda_stream])
            gm.replay()
            torch.cuda.synchronize()
            res[name + "_graph_us"] = round(timed(lambda: gm.replay(), n=50, warm=5) / 100, 3)
            del gm
        except RuntimeError as e:
            res[name + "_graph_error"] = str(e)[:200]
            torch.cuda.synchronize()
        mp.close()
        m.close()
    # CRC32C_MULTI_PIPELINE: consecutive steps into rotating root arrays
    # overlap (step k + 1's shard launch beside step k's tail and gather);
    # joined at the end of the timed steps / inside the capture.
    outs = [torch.zeros(256 * 128, dtype=torch.int32, device=dev) for _ in range(4)]
    for name, flags in (("pipe_in_place", 0), ("pipe_self_send", hdfs.CRC32C_MULTI_SELF_SEND)):
        m = hdfs.Multi([0])
        mp = m.plan(pk, 64, flags | hdfs.CRC32C_MULTI_PIPELINE)
        k = [0]

        def step(sp):
            mp.exec([payload.data_ptr()], outs[k[0] % 4].data_ptr(), [sp])
            k[0] += 1

        def timed_pipe(n=1000, warm=200):
            for _ in range(warm):
                step(stream.cuda_stream)
            mp.join([stream.cuda_stream])
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(n):
                step(stream.cuda_stream)
            mp.join([stream.cuda_stream])
            e1.record(stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / n * 1e3

        res[name + "_us"] = round(timed_pipe(), 3)
        exact = all(np.array_equal(o.cpu().numpy(), out.cpu().numpy()) for o in outs)
        try:
            gm = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gm, stream=cs, capture_error_mode="thread_local"):
                for _ in range(100):
                    step(cs.cuda_stream)
                mp.join([cs.cuda_stream])
            gm.replay()
            torch.cuda.synchronize()
            res[name + "_graph_us"] = round(timed(lambda: gm.replay(), n=50, warm=5) / 100, 3)
            exact = exact and all(np.array_equal(o.cpu().numpy(), out.cpu().numpy()) for o in outs)
            del gm
        except RuntimeError as e:
            res[name + "_graph_error"] = str(e)[:200]
            torch.cuda.synchronize()
        res[name + "_exact"] = exact
        mp.close()
        m.close()
    # One rank of config 4 at N = 8 checksums 4 of the 32 blocks (this shard)
    # and, at rank 0, receives 7 peers' 4 x 32 KiB; a peer's transfer costs at
    # least what the self-send adds to the in-place step (one RCCL group).
    res["gather_lower_bound_us"] = round(res["multi_self_send_us"] - res["multi_in_place_us"], 3)
    res["model_step_n8_us"] = round(res["shard_eager_us"] + res["gather_lower_bound_us"], 3)
    res["model_value_n8_gib_s"] = round(32 * (4 << 20) / (res["model_step_n8_us"] * 1e-6) / 2**30, 1)
    if "pipe_self_send_graph_us" in res:  # (pipelined steps with a gather: measured slower, not used)
        res["model_step_n8_pipe_graph_us"] = res["pipe_self_send_graph_us"]
        res["model_value_n8_pipe_graph_gib_s"] = round(32 * (4 << 20) / (res["pipe_self_send_graph_us"] * 1e-6)
                                                       / 2**30, 1)
    if "multi_self_send_graph_us" in res:  # the bench's config-4 steps are graph-replayed
        res["gather_lower_bound_graph_us"] = round(res["multi_self_send_graph_us"] - res["shard_graph_us"], 3)
        res["model_step_n8_graph_us"] = res["multi_self_send_graph_us"]
        res["model_value_n8_graph_gib_s"] = round(32 * (4 << 20) / (res["multi_self_send_graph_us"] * 1e-6) / 2**30, 1)
    if "multi_self_send_4x_graph_us" in res:  # the same with one N = 8 peer's four ranges (packed)
        res["model_step_n8_graph_4x_us"] = res["multi_self_send_4x_graph_us"]
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
