"""Synthetic batches of the BASELINE.json configs:
packet descriptor arrays and payload bytes for bench.py and tools/.

Packets follow the reference's write path: 64 KiB packets (packetsize,
src/hadooprpc.c:830) cut into bytesPerChecksum chunks, checksums written at
out_idx (hadooprpc.c:733-742).  Payload bytes come from numpy's PCG64
generator; nothing here computes a checksum.
"""
from __future__ import annotations

import numpy as np

from . import PACKET_DTYPE

PACKET_BYTES = 65536


def uniform_packets(npkts: int, pkt_len: int = PACKET_BYTES, bpc: int = 512, stride: int | None = None) -> np.ndarray:
    """npkts equal packets back to back (configs 1-4): packet i at i*stride,
    its checksums at i*ceil(len/bpc)."""
    stride = pkt_len if stride is None else stride
    p = np.zeros(npkts, dtype=PACKET_DTYPE)
    per = (pkt_len + bpc - 1) // bpc
    p["payload_off"] = np.arange(npkts, dtype=np.uint64) * np.uint64(stride)
    p["out_idx"] = np.arange(npkts, dtype=np.uint64) * np.uint64(per)
    p["len"] = pkt_len
    p["bpc"] = bpc
    return p


def mixed_packets(npkts: int, pkt_len: int = PACKET_BYTES, bpcs=(512, 1024, 4096)) -> np.ndarray:
    """Config 5: packets cycling bytesPerChecksum, checksums by prefix sum."""
    p = np.zeros(npkts, dtype=PACKET_DTYPE)
    bpc = np.array([bpcs[i % len(bpcs)] for i in range(npkts)], dtype=np.uint64)
    per = (pkt_len + bpc - 1) // bpc
    p["payload_off"] = np.arange(npkts, dtype=np.uint64) * np.uint64(pkt_len)
    p["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    p["len"] = pkt_len
    p["bpc"] = bpc.astype(np.uint32)
    return p


def config_packets(name: str):
    """(packet descriptors, workload text) of one rank's batch of a
    BASELINE.json config (config 4 is laid out by shard.py)."""
    if name == "c2":
        return uniform_packets(4096), "4096 x 64KiB packets, 512B chunks (BASELINE config 2)"
    if name == "c3":
        return uniform_packets(64), "one 4MiB block as 64 x 64KiB packets, 512B chunks (config 3)"
    if name == "c4":
        return None, "128MiB file as 32 x 4MiB blocks round-robin over ranks (config 4)"
    if name == "c5":
        return mixed_packets(4096), "4096 x 64KiB packets, bpc cycling 512/1024/4096 (config 5)"
    if name == "c2u":  # config 2 with every packet 5 bytes off 16-byte alignment (general path)
        pk = uniform_packets(4096, stride=PACKET_BYTES + 16)
        pk["payload_off"] += np.uint64(5)
        return pk, "4096 x 64KiB packets at 16-byte-misaligned offsets, 512B chunks (general path)"
    if name == "c3u":  # config 3 with every packet 5 bytes off 16-byte alignment
        pk = uniform_packets(64, stride=PACKET_BYTES + 16)
        pk["payload_off"] += np.uint64(5)
        return pk, "one 4MiB block as 64 x 64KiB packets at 16-byte-misaligned offsets, 512B chunks"
    if name == "c2b1536":  # config 2 with bytesPerChecksum 1536 (not a power of two: general path)
        return uniform_packets(4096, bpc=1536), "4096 x 64KiB packets, 1536B chunks (general path)"
    if name == "c2b1000":  # config 2 with bytesPerChecksum 1000 (padded general tiles)
        return uniform_packets(4096, bpc=1000), "4096 x 64KiB packets, 1000B chunks (padded general tiles)"
    if name.startswith("c2w") and name[3:].isdigit():  # chunk-aligned packets: whole chunks, no tail
        bpc = int(name[3:])
        plen = PACKET_BYTES // bpc * bpc
        return (uniform_packets(4096, pkt_len=plen, stride=PACKET_BYTES, bpc=bpc),
                "4096 x %dB packets (%d whole %dB chunks each, 64KiB stride)" % (plen, plen // bpc, bpc))
    if name.startswith("c2b") and name[3:].isdigit():  # config 2 with any other bytesPerChecksum
        bpc = int(name[3:])
        return uniform_packets(4096, bpc=bpc), "4096 x 64KiB packets, %dB chunks (general path)" % bpc
    if name == "c2t":  # config 2 with a 412-byte tail chunk in every packet (4096 general-path items)
        return (uniform_packets(4096, pkt_len=PACKET_BYTES - 100, stride=PACKET_BYTES),
                "4096 x (64KiB - 100 B) packets, 512B chunks + a 412 B tail each")
    if name.startswith("p") and name[1:].isdigit():  # pN: N uniform packets
        n = int(name[1:])
        return uniform_packets(n), "%d x 64KiB packets, 512B chunks" % n
    raise ValueError("unknown config " + name)


def synthetic_bytes(nbytes: int, seed: int) -> np.ndarray:
    """Uniform random payload bytes (PCG64, reproducible per seed)."""
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, size=nbytes, dtype=np.uint8)
