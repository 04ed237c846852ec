"""Python mirror of the multi-GPU layout and gather.

The product path is the C ABI's crc32c_multi_plan_* (csrc/crc32c_multi.hip):
a file's packets dealt round-robin over the ranks in groups of consecutive
packets (one HDFS block each, src/fuse.c:580-647 / src/hadooprpc.c:815-860),
every rank checksumming its shard from its own HBM, and one group of RCCL
point-to-point transfers landing every group's u32 checksum range in file
order on rank 0 -- the path's only exchange.  This module uses the SAME
layout code (crc32c_multi_layout / crc32c_multi_shard_packets, host-only C)
and the same per-group send / receive pattern over torch.distributed, so the
CPU tests can run the N > 1 path under gloo.
"""
from __future__ import annotations

import numpy as np

BLOCK_BYTES = 4 << 20      # dfs.block.size in BASELINE config 3/4
PACKET_BYTES = 64 << 10    # packetsize, src/hadooprpc.c:830


def _pkg():
    import sys

    return sys.modules["hdfs_crc32c_amd"]


def rank_blocks(nblocks: int, world: int, rank: int) -> list[int]:
    """Global block (group) indices owned by `rank` (round-robin)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank %d of world %d" % (rank, world))
    return list(range(rank, nblocks, world))


def layout(pkts, group_packets: int, world: int):
    """(per-group [rank, shard offset, payload offset, bytes], shard bytes per rank) -- crc32c_multi_layout."""
    return _pkg().multi_layout(pkts, group_packets, world)


def rank_payload(file_bytes: np.ndarray, lay: np.ndarray, shard_bytes: np.ndarray, rank: int) -> np.ndarray:
    """Rank's shard buffer, laid out as crc32c_multi_layout says (+16 bytes slack)."""
    out = np.zeros(int(shard_bytes[rank]) + 16, np.uint8)
    for r, soff, poff, n in lay.astype(np.int64):
        if r == rank:
            out[soff:soff + n] = file_bytes[poff:poff + n]
    return out


def rank_packets(pkts, group_packets: int, world: int, rank: int) -> np.ndarray:
    """Rank's packets: payload offsets into its shard, out indices global -- crc32c_multi_shard_packets."""
    return _pkg().multi_shard_packets(pkts, group_packets, world, rank)


def group_ranges(pkts, group_packets: int) -> list[tuple[int, int]]:
    """Each group's checksum range (first global out index, count)."""
    pkts = np.asarray(pkts)
    out = []
    for g in range(0, pkts.size, group_packets):
        p = pkts[g:g + group_packets]
        p = p[p["len"] > 0]
        if not p.size:
            out.append((0, 0))
            continue
        n = (p["len"].astype(np.int64) + p["bpc"] - 1) // p["bpc"]
        out.append((int(p["out_idx"].min()), int(n.sum())))
    return out


def gather_checksums(local, pkts, group_packets: int, world: int, rank: int):
    """Every group's checksum range from its rank's array (a torch int32
    tensor indexed by GLOBAL out index, on the rank's device for nccl or on
    the CPU for gloo) into place on rank 0, one send / receive per group, as
    crc32c_multi_plan_exec does with RCCL.  Returns the file's checksums
    (np.uint32) on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist

    ranges = group_ranges(pkts, group_packets)
    total = max((o + n for o, n in ranges), default=0)
    full = torch.zeros(max(total, 1), dtype=torch.int32, device=local.device) if rank == 0 else None
    ops = []
    for g, (o, n) in enumerate(ranges):
        owner = g % world
        if not n:
            continue
        if owner == rank and rank == 0:
            full[o:o + n] = local[o:o + n]
        elif owner == rank:
            ops.append(dist.P2POp(dist.isend, local[o:o + n].contiguous(), 0))
        elif rank == 0:
            buf = torch.empty(n, dtype=torch.int32, device=local.device)
            ops.append((dist.P2POp(dist.irecv, buf, owner), o, buf))
    if world > 1:
        p2p = [op if isinstance(op, dist.P2POp) else op[0] for op in ops]
        if p2p:
            for req in dist.batch_isend_irecv(p2p):
                req.wait()
        if rank == 0:
            for op in ops:
                if not isinstance(op, dist.P2POp):
                    _, o, buf = op
                    full[o:o + buf.numel()] = buf
    if rank != 0:
        return None
    return full[:total].cpu().numpy().view(np.uint32)
