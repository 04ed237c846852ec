"""N > 1 path on CPU: world-size 2, 3 and 8 process groups over gloo.

The multi-GPU plan deals a file's blocks (groups of
consecutive packets) round-robin over the ranks; each rank checksums its
shard into one local u32 array and sends it to rank 0 -- whole, into a
staging array that rank 0 scatters into file order (the packed gather, when
a sender has several group ranges), or range by range straight into place
-- the path's only exchange.  Every part of that exchange that only N > 1
reaches is the library's own code here: each rank's shard and the packets
its plan computes (payload offsets into the shard, out indices into its
local array) come from crc32c_multi_layout / crc32c_multi_rank_packets, and
what both sides post from crc32c_multi_transfers / crc32c_multi_scatter --
the same host code crc32c_multi_plan_create builds its exec from.  The checksums themselves come from the oracle
(the GPU ranks run the HIP kernel); the transfers are gloo send / receive in
place of RCCL's.  Rank 0's assembled array must equal the reference's golden
digest of config 4's 128 MiB file, or the oracle over the whole file, bit for
bit.  The bench's max-over-ranks timing reduction is checked the same way.
"""
from __future__ import annotations

import hashlib
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN, load_package

PKTS_PER_BLOCK = 4  # 256 KiB blocks keep the CPU oracle fast; the layout is size-independent
PKT = 65536
SELF_SEND = 0x10  # CRC32C_MULTI_SELF_SEND
PER_GROUP = 0x80  # CRC32C_MULTI_PER_GROUP_RECV


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _file_packets(nblocks: int, bpc: int, ragged: bool):
    import oracle

    pk = oracle.uniform_packets(PKTS_PER_BLOCK * nblocks, PKT, bpc)
    if ragged:  # a short last packet in every block and a 5-byte skew in block 1
        pk["len"][PKTS_PER_BLOCK - 1::PKTS_PER_BLOCK] = PKT - 1000
        if nblocks > 1:
            pk["payload_off"][PKTS_PER_BLOCK:2 * PKTS_PER_BLOCK] += 5
            pk["len"][2 * PKTS_PER_BLOCK - 1] -= 5
        per = (pk["len"].astype(np.int64) + pk["bpc"] - 1) // pk["bpc"]
        pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    return pk


def _c4_spec():
    with open(os.path.join(GOLDEN, "batches.json")) as f:
        return [b for b in json.load(f) if b["name"] == "c4_file_128MiB"][0]


def _worker(rank: int, world: int, port: int, case: tuple, flags: int, result_path: str):
    import torch
    import torch.distributed as dist

    import oracle

    load_package().lib()
    from hdfs_crc32c_amd import shard

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        if case[0] == "c4":  # config 4: 32 x 4 MiB blocks of 64 packets, the reference's golden digest
            spec = _c4_spec()
            gp = 64
            pk = oracle.uniform_packets(spec["packets"]["count"], spec["packets"]["len"][0], 512)
            file_bytes = oracle.xorshift64_bytes(spec["payload_bytes"], spec["seed"])
        else:
            _, nblocks, bpc, ragged = case
            gp = PKTS_PER_BLOCK
            pk = _file_packets(nblocks, bpc, ragged)
            file_bytes = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 16, oracle.SEED)
        total = oracle.total_checksums(pk)
        lay, sb = shard.layout(pk, gp, world)
        assert set(int(x) for x in lay[:, 0]) <= set(range(world))
        payload = shard.rank_payload(file_bytes, lay, sb, rank)
        ln, xs = shard.transfers(pk, gp, world, flags)
        mine = shard.plan_packets(pk, gp, world, rank, flags)
        in_place = rank == 0 and not ln[0]
        nlocal = total if in_place else int(ln[rank])
        # the rank's plan output: its chunks at the indices the library's plan uses
        local = oracle.Oracle().batch(payload, mine, max(nlocal, 1)) if mine.size else np.zeros(1, np.uint32)
        if not in_place:
            assert mine.size == 0 or oracle.total_checksums(mine) == nlocal  # the local array is dense
        got = shard.gather_checksums(torch.from_numpy(local.view(np.int32).copy()), pk, gp, world, rank, flags)

        # bench.py's timing rule: the slowest rank's time is the job's
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)

        if rank == 0:
            if case[0] == "c4":
                ok = hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == spec["sha256_le"]
            else:
                ok = bool(np.array_equal(got, oracle.Oracle().batch(file_bytes, pk, total)))
            # the transfers and rank 0's in-place groups cover every checksum exactly once
            seen = np.zeros(total, np.int32)
            for _, _, dst, n in xs.astype(np.int64):
                seen[dst:dst + n] += 1
            if in_place:
                for p in mine:
                    n = (int(p["len"]) + int(p["bpc"]) - 1) // int(p["bpc"])
                    seen[int(p["out_idx"]):int(p["out_idx"]) + n] += 1
            ok = ok and bool(np.all(seen == 1)) and float(t.item()) == float(world)
            with open(result_path, "w") as f:
                f.write("ok" if ok else "mismatch")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,case,flags", [
    (2, ("c4",), 0), (3, ("c4",), 0), (8, ("c4",), 0), (8, ("c4",), SELF_SEND), (8, ("c4",), PER_GROUP),
    (2, ("f", 7, 512, False), 0), (2, ("f", 2, 4096, True), SELF_SEND), (3, ("f", 8, 512, True), 0),
    (2, ("f", 1, 512, False), 0), (3, ("f", 5, 1536, True), 0), (3, ("f", 5, 1536, True), SELF_SEND),
    (8, ("f", 11, 512, True), 0)])
def test_library_transfers_match_reference(tmp_path, world, case, flags):
    import oracle

    oracle.build()
    res = str(tmp_path / "result")
    mp.start_processes(_worker, args=(world, _free_port(), case, flags, res), nprocs=world, join=True,
                       start_method="spawn")
    with open(res) as f:
        assert f.read() == "ok"


def test_transfers_shape():
    """crc32c_multi_transfers on config 4 at 8 ranks: 7 sending ranks of 4
    blocks (32 768 checksums = 128 KiB local arrays), one transfer of 8192
    checksums per block (28), each straight to its block's file index; rank 0
    in place sends nothing.  With CRC32C_MULTI_SELF_SEND rank 0 sends too (32
    transfers); on a one-rank communicator the self-send is ONE transfer
    (consecutive groups merge)."""
    hdfs = load_package()
    hdfs.lib()
    import oracle
    from hdfs_crc32c_amd import shard

    pk = oracle.uniform_packets(2048, 65536, 512)
    ln, xs = shard.transfers(pk, 64, 8)
    assert list(ln) == [0] + [32768] * 7
    assert xs.shape == (28, 4) and set(xs[:, 3]) == {8192}
    # block g (on rank g % 8 > 0) lands at file index 8192 g from local index (g // 8) * 8192
    for r, lo, fo, n in xs.astype(np.int64):
        g = fo // 8192
        assert g % 8 == r and r > 0 and lo == (g // 8) * 8192
    # posting order: for every sender, its transfers in file order
    for r in range(1, 8):
        mine = xs[xs[:, 0] == r]
        assert np.all(np.diff(mine[:, 2].astype(np.int64)) > 0)
    ln, xs = shard.transfers(pk, 64, 8, SELF_SEND)
    assert list(ln) == [32768] * 8 and xs.shape == (32, 4)
    p0 = shard.plan_packets(pk, 64, 8, 0, SELF_SEND)
    assert p0.size == 256 and int(p0["out_idx"].max()) == 32768 - 128  # local indices when self-sending
    assert int(shard.plan_packets(pk, 64, 8, 0)["out_idx"].max()) == 2048 * 128 - 128 - 7 * 64 * 128  # global
    ln, xs = shard.transfers(pk, 64, 1, SELF_SEND)
    assert list(ln) == [262144] and xs.tolist() == [[0, 0, 0, 262144]]
    ln, xs = shard.transfers(pk, 64, 1)
    assert list(ln) == [0] and xs.shape == (0, 4)


def test_packed_gather_layout():
    """crc32c_multi_scatter on config 4 at 8 ranks: each of the 7 senders has
    4 placements 8 blocks apart, so the gather is packed -- rank r's whole
    128 KiB local array lands at staging index 32768 (r - 1), and 224 tiles
    of 1024 checksums copy every block into its file place, covering the
    file's peer blocks exactly once; with CRC32C_MULTI_SELF_SEND rank 0's
    array comes first.  Not packed: one placement per sender (N = 1
    self-send, or groups of 8 blocks at N = 4), or CRC32C_MULTI_PER_GROUP_RECV."""
    hdfs = load_package()
    hdfs.lib()
    import oracle
    from hdfs_crc32c_amd import shard

    pk = oracle.uniform_packets(2048, 65536, 512)
    so, ts = shard.scatter(pk, 64, 8)
    assert list(so) == [0] + [32768 * (r - 1) for r in range(1, 8)]
    assert ts.shape == (224, 3) and set(ts[:, 2]) == {1024}
    seen = np.zeros(2048 * 128, np.int32)
    for src, dst, n in ts.astype(np.int64):
        seen[dst:dst + n] += 1
        g = dst // 8192  # block g of rank g % 8: its local index (g // 8) * 8192 + (dst % 8192)
        assert src == 32768 * (g % 8 - 1) + (g // 8) * 8192 + dst % 8192
    assert np.array_equal(seen.reshape(32, 8192).max(axis=1), np.array([0 if g % 8 == 0 else 1 for g in range(32)]))
    so, ts = shard.scatter(pk, 64, 8, SELF_SEND)
    assert list(so) == [32768 * r for r in range(8)] and ts.shape == (256, 3)
    assert shard.scatter(pk, 64, 8, PER_GROUP)[1].shape == (0, 3)
    assert shard.scatter(pk, 64, 1, SELF_SEND)[1].shape == (0, 3)
    assert shard.scatter(pk, 512, 4)[1].shape == (0, 3)  # (group g on rank g: one range each)


def test_layout_helpers():
    """crc32c_multi_layout / crc32c_multi_shard_packets: groups dealt
    round-robin, each rank's shard its groups back to back with their 16-byte
    phase kept, its packets rebased into the shard with global out indices;
    a group whose checksums are not one contiguous range is refused."""
    hdfs = load_package()
    hdfs.lib()
    import oracle
    from hdfs_crc32c_amd import shard

    assert shard.rank_blocks(32, 8, 3) == [3, 11, 19, 27]
    with pytest.raises(ValueError):
        shard.rank_blocks(4, 2, 2)
    pk = _file_packets(7, 512, True)
    lay, sb = shard.layout(pk, PKTS_PER_BLOCK, 3)
    assert lay.shape == (7, 4) and list(lay[:, 0]) == [g % 3 for g in range(7)]
    for r in range(3):
        rows = lay[lay[:, 0] == r].astype(np.int64)
        ends = rows[:, 1] + rows[:, 3]
        assert np.all(rows[1:, 1] >= ends[:-1]) and int(sb[r]) == int(ends[-1])
        assert np.all(rows[:, 1] % 16 == rows[:, 2] % 16)
        mine = shard.rank_packets(pk, PKTS_PER_BLOCK, 3, r)
        assert mine.size == PKTS_PER_BLOCK * len(shard.rank_blocks(7, 3, r))
        assert np.all(mine["payload_off"] + mine["len"] <= sb[r])
    # the union of the ranks' out indices is every checksum once
    seen = np.zeros(oracle.total_checksums(pk), np.int32)
    for r in range(3):
        for p in shard.rank_packets(pk, PKTS_PER_BLOCK, 3, r):
            n = (int(p["len"]) + int(p["bpc"]) - 1) // int(p["bpc"])
            seen[int(p["out_idx"]):int(p["out_idx"]) + n] += 1
    assert np.all(seen == 1)
    bad = pk.copy()
    bad["out_idx"][1] += 7  # a hole inside group 0
    with pytest.raises(hdfs.Crc32cError):
        shard.layout(bad, PKTS_PER_BLOCK, 2)


# ---- bench.py's rank-consistent graph capture (native-hdfs-fuse_amd/graphs.py) --
def _capture_worker(rank: int, world: int, port: int, fail_rank: int, probe_fail_rank: int, result_path: str):
    import torch.distributed as dist

    load_package()
    from hdfs_crc32c_amd.graphs import capture_agreed

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        calls = {"probe": 0, "capture": 0, "abandon": 0}

        def probe():
            calls["probe"] += 1
            if rank == probe_fail_rank:
                raise RuntimeError("probe capture failed on purpose")

        def capture():
            calls["capture"] += 1
            return {"graph": rank}

        def abandon():  # bench.py rebuilds the communicator here: a collective every rank joins
            calls["abandon"] += 1
            dist.barrier()

        got, err = capture_agreed(capture, world, None, probe=probe, on_abandon=abandon,
                                  inject_fail=(rank == fail_rank))
        with open("%s.%d" % (result_path, rank), "w") as f:
            json.dump({"got": got, "err": err, "calls": calls}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_rank,probe_fail_rank", [(2, -1, -1), (2, 1, -1), (3, 0, -1), (3, -1, 2)])
def test_capture_fallback_is_rank_consistent(tmp_path, world, fail_rank, probe_fail_rank):
    """bench.py's graph capture of a step holding RCCL calls (config 4's
    crc32c_multi_plan_exec) is agreed over the ranks: a step-capture failure
    injected on ONE rank (BENCH_CAPTURE_FAIL_RANK's hook) makes EVERY rank drop
    its graphs, run the communicator rebuild together and issue from the host;
    a probe failure (no collective captured yet) stops every rank before any
    step capture; with no failure every rank keeps its own graph."""
    res = str(tmp_path / "r")
    mp.start_processes(_capture_worker, args=(world, _free_port(), fail_rank, probe_fail_rank, res), nprocs=world,
                       join=True, start_method="spawn")
    out = []
    for r in range(world):
        with open("%s.%d" % (res, r)) as f:
            out.append(json.load(f))
    for r, d in enumerate(out):
        assert d["calls"]["probe"] == 1
        if probe_fail_rank >= 0:
            assert d["got"] is None and d["calls"]["capture"] == 0 and d["calls"]["abandon"] == 0
            assert ("probe" in d["err"]) if r == probe_fail_rank else ("another rank" in d["err"])
        elif fail_rank >= 0:
            assert d["got"] is None and d["calls"]["abandon"] == 1, d
            assert ("injected" in d["err"]) if r == fail_rank else ("another rank" in d["err"])
        else:
            assert d["got"] == {"graph": r} and d["err"] is None and d["calls"]["abandon"] == 0
