"""Python mirror of the multi-GPU layout and gather.

The product path is the C ABI's crc32c_multi_plan_* (csrc/crc32c_multi.hip):
a file's packets dealt round-robin over the ranks in groups of consecutive
packets (one HDFS block each, src/fuse.c:580-647 / src/hadooprpc.c:815-860),
every rank checksumming its shard from its own HBM, and one group of RCCL
point-to-point transfers landing every group's u32 checksum range in file
order on rank 0 -- the path's only exchange.  This module uses the SAME
layout code (crc32c_multi_layout / crc32c_multi_shard_packets /
crc32c_multi_transfers / crc32c_multi_scatter, host-only C) and the same
send / receive pattern over torch.distributed, so the CPU tests can run the
N > 1 path under gloo.
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


def plan_packets(pkts, group_packets: int, world: int, rank: int, flags: int = 0) -> np.ndarray:
    """The packets rank's plan computes: payload offsets into its shard, out
    indices into the array it sends to rank 0 (rank 0: global, in place,
    unless CRC32C_MULTI_SELF_SEND) -- crc32c_multi_rank_packets."""
    return _pkg().multi_rank_packets(pkts, group_packets, world, rank, flags)


def transfers(pkts, group_packets: int, world: int, flags: int = 0):
    """(local_nout, transfers {sending rank, local index, file index, count}) -- crc32c_multi_transfers."""
    return _pkg().multi_transfers(pkts, group_packets, world, flags)


def scatter(pkts, group_packets: int, world: int, flags: int = 0):
    """(stage_off, tiles {staging index, file index, count}) of the packed gather -- crc32c_multi_scatter."""
    return _pkg().multi_scatter(pkts, group_packets, world, flags)


def gather_checksums(local, pkts, group_packets: int, world: int, rank: int, flags: int = 0):
    """The exchange of crc32c_multi_plan_exec, over torch.distributed: `local`
    is the u32 array this rank's plan wrote (a torch int32 tensor laid out by
    plan_packets -- rank 0's in place, indexed by global out index, unless
    CRC32C_MULTI_SELF_SEND).  The library's lists drive it exactly as they
    drive the RCCL group.  Packed (crc32c_multi_scatter has tiles: some
    sender has several placements): every sender sends its whole local array
    once, rank 0 receives each into its staging array at stage_off[sender]
    and copies every tile into file order (the scatter kernel's work).
    Otherwise every sender sends each of its transfers' local ranges, in list
    order, and rank 0 receives each straight into its file-order place.
    Returns the file's checksums (np.uint32) on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist

    ln, xs = transfers(pkts, group_packets, world, flags)
    so, ts = scatter(pkts, group_packets, world, flags)
    total = int(_pkg().total_checksums(pkts))
    ops = []
    full = None
    if rank == 0:
        full = torch.zeros(max(total, 1), dtype=torch.int32, device=local.device)
        if not ln[0]:  # rank 0 in place: its own groups are already at their file indices
            full[:min(total, local.numel())] = local[:total]
    if ts.shape[0]:
        senders = [r for r in range(world) if ln[r]]
        stage = None
        if rank == 0:
            stage = torch.zeros(max(int(sum(int(ln[r]) for r in senders)), 1), dtype=torch.int32, device=local.device)
        for r in senders:
            lo, n = int(so[r]), int(ln[r])
            if r == rank and rank == 0:  # self-send
                stage[lo:lo + n] = local[:n]
            elif r == rank:
                ops.append(dist.P2POp(dist.isend, local[:n].contiguous(), 0))
            elif rank == 0:
                ops.append(dist.P2POp(dist.irecv, stage[lo:lo + n], int(r)))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if rank != 0:
            return None
        for src, dst, n in ts.astype(np.int64):
            full[dst:dst + n] = stage[src:src + n]
        return full[:total].cpu().numpy().view(np.uint32)
    for r, lo, fo, n in xs.astype(np.int64):
        if r == rank and rank == 0:  # self-send: RCCL copies rank 0's range into its own output
            full[fo:fo + n] = local[lo:lo + n]
        elif r == rank:
            ops.append(dist.P2POp(dist.isend, local[lo:lo + n].contiguous(), 0))
        elif rank == 0:
            ops.append(dist.P2POp(dist.irecv, full[fo:fo + n], int(r)))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank != 0:
        return None
    return full[:total].cpu().numpy().view(np.uint32)
