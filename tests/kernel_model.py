"""Bit-level numpy model of the HIP kernel's arithmetic (test infrastructure).

It reads the SAME LDS image and constants the library uploads to the GPU
(``crc32c_debug_lds_image``) and evaluates them the way
``crc32c_kernel.hip`` does -- positional nibble lookups per 16-byte lane
piece, XOR over the 32 lanes of a 512-byte block, Z^(512 s) shifts across the
blocks of a chunk, zero-prefixed virtual blocks + Horner for general chunks --
so the CPU suite can check the table layout and the algebra against the
oracle without a GPU.  The GPU suite then checks the kernel itself.
"""
from __future__ import annotations

import numpy as np

LDS_SHIFT_OFF = 65536


class KernelModel:
    def __init__(self, img: np.ndarray, c_lg: np.ndarray, c_small: np.ndarray):
        self.w = img.view("<u4")
        self.c_lg = [int(x) for x in c_lg]
        self.c_small = [int(x) for x in c_small]
        q = np.arange(32)[:, None]
        k = np.arange(16)[None, :]
        n = np.arange(16)[:, None, None]
        # lo[n, q, k] / hi[n, q, k]: table entries addressed as the kernel does
        self.lo = self.w[((k * 4096 + n * 256 + q * 4) // 4)]
        self.hi = self.w[((128 + k * 256 + n * 4096 + q * 4) // 4)]

    def block_lin(self, blocks: np.ndarray) -> np.ndarray:
        """lin() of each 512-byte block: blocks (B, 512) uint8 -> (B,) uint32."""
        b = blocks.reshape(-1, 32, 16)
        qi = np.arange(32)[None, :, None]
        ki = np.arange(16)[None, None, :]
        v = self.lo[b & 15, qi, ki] ^ self.hi[b >> 4, qi, ki]
        return np.bitwise_xor.reduce(v.reshape(v.shape[0], -1), axis=1).astype(np.uint32)

    def zshift(self, s: int, x: int) -> int:
        base = (LDS_SHIFT_OFF + (s - 1) * 512) // 4
        r = 0
        for t in range(8):
            r ^= int(self.w[base + t * 16 + ((x >> (4 * t)) & 15)])
        return r

    def fast_chunks(self, data: np.ndarray, lg: int) -> np.ndarray:
        """Full chunks of 512 << lg bytes, fast-tile arithmetic."""
        nbc = 1 << lg
        lins = self.block_lin(data.reshape(-1, 512)).reshape(-1, nbc)
        out = np.empty(lins.shape[0], np.uint32)
        for c in range(lins.shape[0]):
            x = 0
            for m in range(nbc):
                s = nbc - 1 - m
                x ^= self.zshift(s, int(lins[c, m])) if s else int(lins[c, m])
            out[c] = x ^ self.c_lg[lg]
        return out

    def general_chunk(self, chunk: np.ndarray) -> int:
        """Any length >= 1: FF folded into the first 4 bytes, zero prefix, Horner."""
        r = chunk.size
        nbv = (r + 511) // 512
        pad = nbv * 512 - r
        v = np.zeros(nbv * 512, np.uint8)
        v[pad:] = chunk
        if r >= 4:
            v[pad:pad + 4] ^= 0xFF
        lins = self.block_lin(v.reshape(nbv, 512))
        acc = 0
        for m in range(nbv):
            acc = self.zshift(1, acc) ^ int(lins[m])
        return acc ^ (0xFFFFFFFF if r >= 4 else self.c_small[r])


class KernelModelS4:
    """The slicing-by-4 variants' arithmetic over their LDS image
    (``crc32c_debug_lds_image_s4``): per 16-byte lane piece
    u = S(S(S(d0) ^ d1) ^ d2) ^ d3 from the replicated byte tables, then the
    column operator N_q(u) from 8 nibble lookups; XOR over the 32 lanes."""

    NIB_OFF = 131072
    SHIFT_OFF = 147456

    def __init__(self, img: np.ndarray):
        self.w = img.view("<u4")
        b = np.arange(256)
        q = np.arange(32)
        # t_m[b, q]: byte table m at column q
        self.t = [self.w[((m >> 1) * 65536 + b[:, None] * 256 + (m & 1) * 128 + q[None, :] * 4) // 4]
                  for m in range(4)]
        t = np.arange(8)
        n = np.arange(16)
        # nq[q, t, n]
        self.nq = self.w[(self.NIB_OFF + (t[None, :, None] >> 1) * 4096 + n[None, None, :] * 256
                          + (t[None, :, None] & 1) * 128 + q[:, None, None] * 4) // 4]

    def s(self, u: np.ndarray, q: np.ndarray) -> np.ndarray:
        return (self.t[3][u & 0xFF, q] ^ self.t[2][(u >> 8) & 0xFF, q] ^ self.t[1][(u >> 16) & 0xFF, q]
                ^ self.t[0][(u >> 24) & 0xFF, q])

    def block_lin(self, blocks: np.ndarray) -> np.ndarray:
        d = np.ascontiguousarray(blocks).view("<u4").reshape(-1, 32, 4)
        q = np.broadcast_to(np.arange(32)[None, :], d.shape[:2])
        u = self.s(self.s(self.s(d[..., 0], q) ^ d[..., 1], q) ^ d[..., 2], q) ^ d[..., 3]
        acc = np.zeros(u.shape, np.uint32)
        for t in range(8):
            acc ^= self.nq[q, t, (u >> (4 * t)) & 15]
        return np.bitwise_xor.reduce(acc, axis=1).astype(np.uint32)
