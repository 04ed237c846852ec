"""N > 1 path on CPU: world-size 2 and 3 process groups over gloo.

The multi-GPU layout (native-hdfs-fuse_amd/shard.py)
shards a file's 4 MiB blocks round-robin over the ranks and gathers the
u32 checksum arrays to rank 0 -- the path's only collective.  Here each rank
computes its blocks' checksums with the oracle (the GPU ranks use the HIP
kernel; the layout and the gather are the same code), and rank 0 checks the
assembled array against the oracle over the whole file, bit for bit.  The
bench's max-over-ranks timing reduction is checked the same way.
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


def _worker(rank: int, world: int, port: int, nblocks: int, bpc: int, result_path: str):
    import torch
    import torch.distributed as dist

    import oracle

    hdfs = load_package()
    from hdfs_crc32c_amd import shard

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        block_bytes = PKTS_PER_BLOCK * PKT
        file_bytes = oracle.xorshift64_bytes(nblocks * block_bytes, oracle.SEED)
        blocks = shard.rank_blocks(nblocks, world, rank)
        payload = shard.rank_payload(file_bytes, blocks, block_bytes)
        pk = oracle.uniform_packets(PKTS_PER_BLOCK * len(blocks), PKT, bpc)
        per_block = PKTS_PER_BLOCK * ((PKT + bpc - 1) // bpc)
        orc = oracle.Oracle()
        local = orc.batch(payload, pk, len(blocks) * per_block) if blocks else np.zeros(0, np.uint32)
        got = shard.gather_checksums(torch.from_numpy(local.view(np.int32).copy()), nblocks, per_block, world, rank)

        # bench.py's timing rule: the slowest rank's time is the job's
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)

        if rank == 0:
            whole = oracle.uniform_packets(PKTS_PER_BLOCK * nblocks, PKT, bpc)
            want = orc.batch(file_bytes, whole, nblocks * per_block)
            ok = bool(np.array_equal(got, want)) and float(t.item()) == float(world)
            with open(result_path, "w") as f:
                f.write("ok" if ok else "mismatch")
        assert hdfs is not None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nblocks,bpc", [(2, 7, 512), (2, 2, 4096), (3, 8, 512), (2, 1, 512)])
def test_round_robin_gather_matches_oracle(tmp_path, world, nblocks, bpc):
    import oracle

    oracle.build()
    res = str(tmp_path / "result")
    mp.start_processes(_worker, args=(world, _free_port(), nblocks, bpc, res), nprocs=world, join=True,
                       start_method="spawn")
    with open(res) as f:
        assert f.read() == "ok"


def test_layout_helpers():
    hdfs = load_package()
    from hdfs_crc32c_amd import shard

    assert shard.rank_blocks(32, 8, 3) == [3, 11, 19, 27]
    assert shard.rank_blocks(7, 2, 1) == [1, 3, 5]
    assert shard.max_blocks_per_rank(7, 2) == 4
    # assemble() inverts the round-robin deal, padding included
    per = 3
    world, nblocks = 3, 7
    arrays = []
    for r in range(world):
        bl = shard.rank_blocks(nblocks, world, r)
        a = np.zeros(shard.max_blocks_per_rank(nblocks, world) * per, np.uint32)
        for j, b in enumerate(bl):
            a[j * per:(j + 1) * per] = b * 100 + np.arange(per)
        arrays.append(a)
    full = shard.assemble(arrays, nblocks, per)
    assert np.array_equal(full, (np.arange(nblocks)[:, None] * 100 + np.arange(per)).reshape(-1))
    with pytest.raises(ValueError):
        shard.rank_blocks(4, 2, 2)
    assert hdfs is not None
