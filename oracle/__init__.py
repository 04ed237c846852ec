"""TEST INFRASTRUCTURE ONLY -- the CPU parity oracle for the CRC32C chunk path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package.  The product library
(``native-hdfs-fuse_amd``) never imports, links or calls it.

Two checkers live here:

* ``Oracle`` -- ctypes view of ``crc32c_oracle.c``, a clean-room C
  restatement of ``/root/reference/src/crc32c.c`` (slicing-by-8 and bytewise,
  crc32c.c:43-107) and of the packet writer's chunk loop
  (``src/hadooprpc.c:639, 733-742``) and packetisation (``hadooprpc.c:827-857``).
* ``Reference`` -- ctypes view of ``_ref/libref_crc32c.so``: the UNMODIFIED
  ``/root/reference/src/crc32c.c`` compiled where it lies (``oracle/Makefile``)
  plus ``ref_harness.c``.  It only exists where it was built (this container,
  and GPU boxes that received the built file through gpurun).

``py_crc32c`` is a third, pure-Python bytewise restatement for tiny inputs.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "_build", "liboracle_crc32c.so")
REF_SO = os.path.join(HERE, "_ref", "libref_crc32c.so")
REF_SRC = "/root/reference/src/crc32c.c"

# The synthetic-data seed used by the survey's CPU probe and the fixtures
# (SURVEY.md section 8d).
SEED = 0x9E3779B97F4A7C15
POLY = 0x82F63B78  # crc32c.c:43


class PacketDesc(ctypes.Structure):
    """Mirror of ``crc32c_packet`` in include/hdfs_crc32c.h."""

    _fields_ = [
        ("payload_off", ctypes.c_uint64),
        ("out_idx", ctypes.c_uint64),
        ("len", ctypes.c_uint32),
        ("bpc", ctypes.c_uint32),
    ]


PACKET_DTYPE = np.dtype(
    [("payload_off", "<u8"), ("out_idx", "<u8"), ("len", "<u4"), ("bpc", "<u4")], align=True
)
assert PACKET_DTYPE.itemsize == ctypes.sizeof(PacketDesc) == 24


def build(quiet: bool = True) -> None:
    """Compile the oracle (and the reference harness when the reference tree
    is present).  Building the checker is not using it."""
    out = subprocess.DEVNULL if quiet else None
    subprocess.run(["make", "-C", HERE], check=True, stdout=out)


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def xorshift64_bytes(nbytes: int, seed: int = SEED) -> np.ndarray:
    """Vectorised numpy twin of oracle_xorshift64_fill (same byte stream)."""
    nwords = (nbytes + 7) // 8
    words = np.empty(nwords, dtype=np.uint64)
    s = np.uint64(seed if seed else SEED)
    # The recurrence is sequential; do it in C when the oracle is built.
    lib = _oracle_lib_or_none()
    if lib is not None:
        buf = np.empty(nbytes, dtype=np.uint8)
        lib.oracle_xorshift64_fill(ctypes.c_uint64(int(s)), _ptr(buf), ctypes.c_uint64(nbytes))
        return buf
    m = (1 << 64) - 1
    x = int(s)
    for i in range(nwords):
        x ^= (x << 13) & m
        x ^= x >> 7
        x ^= (x << 17) & m
        words[i] = x
    return words.view(np.uint8)[:nbytes].copy()


_ORACLE_LIB = None


def _oracle_lib_or_none():
    global _ORACLE_LIB
    if _ORACLE_LIB is None and os.path.exists(ORACLE_SO):
        _ORACLE_LIB = _bind_oracle(ctypes.CDLL(ORACLE_SO))
    return _ORACLE_LIB


def _bind_oracle(lib):
    u32, u64, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p
    lib.oracle_crc32c_bytewise.restype = u32
    lib.oracle_crc32c_bytewise.argtypes = [u32, vp, ctypes.c_size_t]
    lib.oracle_crc32c_slice8.restype = u32
    lib.oracle_crc32c_slice8.argtypes = [u32, vp, ctypes.c_size_t]
    lib.oracle_nchunks.restype = u64
    lib.oracle_nchunks.argtypes = [u64, u32]
    lib.oracle_chunks.restype = u64
    lib.oracle_chunks.argtypes = [vp, u64, u32, vp, ctypes.c_int]
    lib.oracle_batch.restype = None
    lib.oracle_batch.argtypes = [vp, vp, u64, vp, ctypes.c_int]
    lib.oracle_packetize.restype = u64
    lib.oracle_packetize.argtypes = [u64, u64, u32, u32, vp, u64]
    lib.oracle_xorshift64_fill.restype = None
    lib.oracle_xorshift64_fill.argtypes = [u64, vp, u64]
    lib.oracle_batch_mt.restype = ctypes.c_double
    lib.oracle_batch_mt.argtypes = [vp, vp, u64, vp, ctypes.c_int, ctypes.c_int]
    return lib


class Oracle:
    """The clean-room C restatement (crc32c_oracle.c)."""

    def __init__(self):
        if not os.path.exists(ORACLE_SO):
            build()
        self.lib = _oracle_lib_or_none()
        if self.lib is None:
            raise RuntimeError("oracle library missing: " + ORACLE_SO)

    def crc32c(self, data, crc: int = 0, bytewise: bool = False) -> int:
        a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        a = np.ascontiguousarray(a, dtype=np.uint8)
        f = self.lib.oracle_crc32c_bytewise if bytewise else self.lib.oracle_crc32c_slice8
        return int(f(crc & 0xFFFFFFFF, _ptr(a), a.size))

    def chunks(self, packet: np.ndarray, bpc: int, big_endian: bool = False) -> np.ndarray:
        packet = np.ascontiguousarray(packet, dtype=np.uint8)
        n = int(self.lib.oracle_nchunks(packet.size, bpc))
        out = np.zeros(max(n, 1), dtype=np.uint32)
        self.lib.oracle_chunks(_ptr(packet), packet.size, bpc, _ptr(out), int(big_endian))
        return out[:n]

    def batch(self, payload: np.ndarray, pkts: np.ndarray, nout: int, big_endian: bool = False) -> np.ndarray:
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        pkts = np.ascontiguousarray(pkts, dtype=PACKET_DTYPE)
        out = np.zeros(max(nout, 1), dtype=np.uint32)
        self.lib.oracle_batch(_ptr(payload), _ptr(pkts), pkts.size, _ptr(out), int(big_endian))
        return out[:nout]

    def packetize(self, length: int, blockoffset: int, packetsize: int, bpc: int) -> list:
        cap = 1 << 16
        lens = np.zeros(cap, dtype=np.uint64)
        n = int(self.lib.oracle_packetize(length, blockoffset, packetsize, bpc, _ptr(lens), cap))
        assert n <= cap
        return [int(x) for x in lens[:n]]

    def batch_mt_seconds(self, payload, pkts, out, nthreads: int, reps: int) -> float:
        return float(self.lib.oracle_batch_mt(_ptr(payload), _ptr(pkts), pkts.size, _ptr(out), nthreads, reps))


class Reference:
    """The reference's own crc32c.c (compiled where it lies, never copied)."""

    def __init__(self):
        if not os.path.exists(REF_SO):
            if os.path.exists(REF_SRC):
                build()
            if not os.path.exists(REF_SO):
                raise FileNotFoundError(REF_SO)
        lib = ctypes.CDLL(REF_SO)
        u32, u64, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p
        lib.ref_crc32c.restype = u32
        lib.ref_crc32c.argtypes = [u32, vp, ctypes.c_size_t]
        lib.ref_batch.restype = None
        lib.ref_batch.argtypes = [vp, vp, u64, vp]
        lib.ref_batch_mt.restype = ctypes.c_double
        lib.ref_batch_mt.argtypes = [vp, vp, u64, vp, ctypes.c_int, ctypes.c_int]
        lib.ref_batch_mt_rot.restype = ctypes.c_double
        lib.ref_batch_mt_rot.argtypes = [vp, u64, vp, u64, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        lib.ref_block_latency.restype = ctypes.c_double
        lib.ref_block_latency.argtypes = [vp, vp, u64, vp, ctypes.c_int, ctypes.c_int]
        self.lib = lib

    @staticmethod
    def available() -> bool:
        return os.path.exists(REF_SO) or os.path.exists(REF_SRC)

    def crc32c(self, data, crc: int = 0) -> int:
        a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        a = np.ascontiguousarray(a, dtype=np.uint8)
        return int(self.lib.ref_crc32c(crc & 0xFFFFFFFF, _ptr(a), a.size))

    def batch(self, payload: np.ndarray, pkts: np.ndarray, nout: int) -> np.ndarray:
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        pkts = np.ascontiguousarray(pkts, dtype=PACKET_DTYPE)
        out = np.zeros(max(nout, 1), dtype=np.uint32)
        self.lib.ref_batch(_ptr(payload), _ptr(pkts), pkts.size, _ptr(out))
        return out[:nout]

    def batch_mt_seconds(self, payload, pkts, out, nthreads: int, reps: int) -> float:
        return float(self.lib.ref_batch_mt(_ptr(payload), _ptr(pkts), pkts.size, _ptr(out), nthreads, reps))

    def block_latency_seconds(self, payload, pkts, out, nthreads: int, reps: int) -> float:
        """Mean wall seconds of one call over the batch split over nthreads
        persistent threads (ref_harness.c ref_block_latency; in-cache)."""
        return float(self.lib.ref_block_latency(_ptr(payload), _ptr(pkts), pkts.size, _ptr(out), nthreads, reps))

    def batch_rot_seconds(self, payload, pkts, out, nthreads: int, nbuf: int, reps: int) -> float:
        """Full-width timing: nbuf distinct first-touched copies rotated over reps
        (ref_harness.c ref_batch_mt_rot); wall seconds of the reps."""
        t = float(self.lib.ref_batch_mt_rot(_ptr(payload), payload.size, _ptr(pkts), pkts.size, _ptr(out), nthreads,
                                            nbuf, reps))
        if t < 0:
            raise MemoryError("ref_batch_mt_rot: allocation failed")
        return t


def py_crc32c(data: bytes, crc: int = 0) -> int:
    """Pure-Python bitwise restatement (crc32c.c:43, 56-63, 84, 106); tiny inputs only."""
    r = (~crc) & 0xFFFFFFFF
    for b in bytes(data):
        r ^= b
        for _ in range(8):
            r = (r >> 1) ^ (POLY if (r & 1) else 0)
    return (~r) & 0xFFFFFFFF


def uniform_packets(npkts: int, pkt_len: int = 65536, bpc: int = 512, stride: int | None = None) -> np.ndarray:
    """Contiguous batch of equal packets (configs 1-4): packet i at i*stride,
    checksums at i*ceil(len/bpc)."""
    stride = pkt_len if stride is None else stride
    p = np.zeros(npkts, dtype=PACKET_DTYPE)
    per = (pkt_len + bpc - 1) // bpc
    p["payload_off"] = np.arange(npkts, dtype=np.uint64) * np.uint64(stride)
    p["out_idx"] = np.arange(npkts, dtype=np.uint64) * np.uint64(per)
    p["len"] = pkt_len
    p["bpc"] = bpc
    return p


def mixed_packets(npkts: int, pkt_len: int = 65536, bpcs=(512, 1024, 4096)) -> np.ndarray:
    """Config 5: packets cycling bytes-per-checksum, outputs by prefix sum."""
    p = np.zeros(npkts, dtype=PACKET_DTYPE)
    bpc = np.array([bpcs[i % len(bpcs)] for i in range(npkts)], dtype=np.uint32)
    per = (pkt_len + bpc.astype(np.uint64) - 1) // bpc.astype(np.uint64)
    p["payload_off"] = np.arange(npkts, dtype=np.uint64) * np.uint64(pkt_len)
    p["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    p["len"] = pkt_len
    p["bpc"] = bpc
    return p


def total_checksums(pkts: np.ndarray) -> int:
    """Length of the checksum array a batch fills: max of out_idx + roundup(len, bpc)
    (hadooprpc.c:639) over the packets with len > 0.  A zero-length packet (the
    block's last-packet marker, hadooprpc.c:644 / 853-856) has no checksums, whatever
    its bpc."""
    pkts = pkts[pkts["len"] > 0]
    if pkts.size == 0:
        return 0
    per = (pkts["len"].astype(np.uint64) + pkts["bpc"].astype(np.uint64) - 1) // pkts["bpc"].astype(np.uint64)
    return int((pkts["out_idx"] + per).max())


# ---- Hadoop CHECKSUM_CRC32 ("next" row 3) ------------
# The reference has no CRC32 implementation (hadooprpc.c:629-631 returns
# -ENOSYS).  Hadoop's CHECKSUM_CRC32 is java.util.zip.CRC32, i.e. zlib's
# crc32; Python's zlib module (the system zlib) is the independent oracle,
# applied per chunk exactly as the CRC32C loop of hadooprpc.c:733-742.
def zlib_chunks(packet: np.ndarray, bpc: int) -> np.ndarray:
    import zlib

    b = np.ascontiguousarray(packet, dtype=np.uint8).tobytes()
    return np.array([zlib.crc32(b[i:i + bpc]) for i in range(0, len(b), bpc)], dtype=np.uint32)


def zlib_batch(payload: np.ndarray, pkts: np.ndarray, nout: int) -> np.ndarray:
    import zlib

    out = np.zeros(max(nout, 1), dtype=np.uint32)
    mv = memoryview(np.ascontiguousarray(payload, dtype=np.uint8))
    for p in pkts:
        off, n, bpc, oi = int(p["payload_off"]), int(p["len"]), int(p["bpc"]), int(p["out_idx"])
        for i, c in enumerate(range(0, n, bpc)):
            out[oi + i] = zlib.crc32(mv[off + c:off + min(c + bpc, n)])
    return out[:nout]
