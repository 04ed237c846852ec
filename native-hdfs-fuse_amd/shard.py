"""Multi-GPU layout of the CRC32C path.

Every chunk's checksum depends only on its own bytes (crc32c(0, chunk),
src/hadooprpc.c:740), and packets / blocks are independent
(src/hadooprpc.c:815-860, src/fuse.c:580-647), so a file shards by whole
blocks with no data-path exchange: block b of the file goes to rank
b mod world (round-robin, as BASELINE config 4 states), each rank checksums
its blocks from its own HBM, and the only collective is one gather of the
u32 checksum arrays to rank 0 (RCCL over xGMI on the GPU box; gloo in the
CPU tests).  One process per GPU.

Functions here are pure host logic plus one torch.distributed call, so the
same code runs under ``gloo`` on CPU tensors and ``nccl`` (= RCCL) on GPU
tensors.
"""
from __future__ import annotations

import numpy as np

BLOCK_BYTES = 4 << 20      # dfs.block.size in BASELINE config 3/4
PACKET_BYTES = 64 << 10    # packetsize, src/hadooprpc.c:830


def rank_blocks(nblocks: int, world: int, rank: int) -> list[int]:
    """Global block indices owned by `rank` (round-robin)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank %d of world %d" % (rank, world))
    return list(range(rank, nblocks, world))


def max_blocks_per_rank(nblocks: int, world: int) -> int:
    return (nblocks + world - 1) // world


def rank_payload(file_bytes: np.ndarray, blocks: list[int], block_bytes: int = BLOCK_BYTES) -> np.ndarray:
    """The rank's device buffer: its blocks back to back (block j of the
    rank at offset j * block_bytes)."""
    out = np.empty(len(blocks) * block_bytes, dtype=np.uint8)
    for j, b in enumerate(blocks):
        out[j * block_bytes:(j + 1) * block_bytes] = file_bytes[b * block_bytes:(b + 1) * block_bytes]
    return out


def assemble(gathered: list[np.ndarray], nblocks: int, per_block: int) -> np.ndarray:
    """Rank 0: the file's checksum array in block order from every rank's
    (padded) array; rank r's j-th block is global block r + j * world."""
    world = len(gathered)
    out = np.empty(nblocks * per_block, dtype=np.uint32)
    for r, arr in enumerate(gathered):
        a = np.asarray(arr).view(np.uint32)
        for j, b in enumerate(range(r, nblocks, world)):
            out[b * per_block:(b + 1) * per_block] = a[j * per_block:(j + 1) * per_block]
    return out


def gather_checksums(local, nblocks: int, per_block: int, world: int, rank: int):
    """Gather every rank's checksum array (a torch int32 tensor holding
    len(rank_blocks) * per_block values, on the rank's device for nccl or on
    the CPU for gloo) to rank 0.  Returns the file's checksums in block
    order (np.uint32) on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist

    cap = max_blocks_per_rank(nblocks, world) * per_block
    send = torch.zeros(cap, dtype=torch.int32, device=local.device)
    n = min(int(local.numel()), cap)
    send[:n] = local.reshape(-1)[:n]
    if world == 1:
        return assemble([send.cpu().numpy()], nblocks, per_block)
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
    dist.gather(send, bufs, dst=0)
    if rank != 0:
        return None
    return assemble([b.cpu().numpy() for b in bufs], nblocks, per_block)
