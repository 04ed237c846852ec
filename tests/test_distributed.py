"""N > 1 path on CPU: world-size 2 and 3 process groups over gloo.

The multi-GPU layout deals a file's blocks (groups of
consecutive packets) round-robin over the ranks and gathers every group's
u32 checksum range to rank 0 -- the path's only exchange.  Each rank here
takes its shard and its packets from the library's own layout code
(crc32c_multi_layout / crc32c_multi_shard_packets, the host half of
crc32c_multi_plan_*), computes their checksums with the oracle (the GPU
ranks run the HIP kernel), and the per-group send / receive of shard.py
(the same pattern crc32c_multi_plan_exec issues through RCCL) lands them on
rank 0, which checks the assembled array against the oracle over the whole
file, bit for bit.  The bench's max-over-ranks timing reduction is checked
the same way.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import load_package

PKTS_PER_BLOCK = 4  # 256 KiB blocks keep the CPU oracle fast; the layout is size-independent
PKT = 65536


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


def _worker(rank: int, world: int, port: int, nblocks: int, bpc: int, ragged: bool, result_path: str):
    import torch
    import torch.distributed as dist

    import oracle

    load_package().lib()
    from hdfs_crc32c_amd import shard

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        pk = _file_packets(nblocks, bpc, ragged)
        total = oracle.total_checksums(pk)
        file_bytes = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 16, oracle.SEED)
        lay, sb = shard.layout(pk, PKTS_PER_BLOCK, world)
        payload = shard.rank_payload(file_bytes, lay, sb, rank)
        mine = shard.rank_packets(pk, PKTS_PER_BLOCK, world, rank)
        assert set(int(x) for x in lay[:, 0]) <= set(range(world))
        orc = oracle.Oracle()
        local = np.zeros(max(total, 1), np.uint32)
        if mine.size:
            local = orc.batch(payload, mine, max(total, 1))  # global out indices, this rank's chunks only
        got = shard.gather_checksums(torch.from_numpy(local.view(np.int32).copy()), pk, PKTS_PER_BLOCK, world,
                                     rank)

        # bench.py's timing rule: the slowest rank's time is the job's
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)

        if rank == 0:
            want = orc.batch(file_bytes, pk, total)
            ok = bool(np.array_equal(got, want)) and float(t.item()) == float(world)
            with open(result_path, "w") as f:
                f.write("ok" if ok else "mismatch")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nblocks,bpc,ragged", [(2, 7, 512, False), (2, 2, 4096, True), (3, 8, 512, True),
                                                      (2, 1, 512, False), (3, 5, 1536, True),
                                                      (8, 32, 512, False), (8, 11, 512, True)])
def test_round_robin_gather_matches_oracle(tmp_path, world, nblocks, bpc, ragged):
    import oracle

    oracle.build()
    res = str(tmp_path / "result")
    mp.start_processes(_worker, args=(world, _free_port(), nblocks, bpc, ragged, res), nprocs=world, join=True,
                       start_method="spawn")
    with open(res) as f:
        assert f.read() == "ok"


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
