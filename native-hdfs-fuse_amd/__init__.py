"""Python view of libhdfs_crc32c.so -- the MI355X CRC32C chunk path of
native-hdfs-fuse, behind the C ABI in ``include/hdfs_crc32c.h``.

The reference is a C program; its interface for this path is the C function
``crc32c(crc, buf, len)`` (``src/crc32c.c:333``) called once per chunk by
``hadoop_rpc_send_packet`` (``src/hadooprpc.c:733-742``).  This module is a
thin ctypes mirror of the C ABI used by the tests and the bench; the product
is the shared library.  No CPU fallback exists for the GPU entry points: if
the library cannot reach a gfx950 device they raise ``Crc32cError``.

Device buffers are passed as raw pointers (``tensor.data_ptr()`` when the
caller uses torch for allocation) and streams as raw ``hipStream_t`` handles
(``torch.cuda.current_stream().cuda_stream``).
"""
from __future__ import annotations

import ctypes
import errno
import numbers
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libhdfs_crc32c.so")
DEBUG_LIB_PATH = os.path.join(HERE, "libhdfs_crc32c_debug.so")  # A/B variants + read probe (tools only)
INCLUDE_DIR = os.path.join(os.path.dirname(HERE), "include")

CRC32C_BIG_ENDIAN = 0x1
CRC32C_TYPE_CRC32 = 0x2  # Hadoop CHECKSUM_CRC32 (zlib polynomial) instead of CRC32C
CRC32C_DEVICE_ADDRESSES = 0x4  # plan flag: payload_off are device addresses; exec/verify take payload 0
CRC32C_CPU_FALLBACK = 0x8  # crc32c_chunks / crc32c_batch_host: finish on the host CPU if the GPU fails
CRC32C_MULTI_SELF_SEND = 0x10  # multi plan: rank 0's own checksums also go through RCCL (one-GPU transport test)
CRC32C_COUNT_COMPLETION = 0x20  # plan: launches count their completion on the GPU; destroy after the streams is safe
CRC32C_MULTI_PIPELINE = 0x40  # multi plan: consecutive execs overlap; results complete after join()
CRC32C_MULTI_PER_GROUP_RECV = 0x80  # multi plan (A/B): one send/recv pair per group range, no packed gather
CRC32C_VERIFY_OVERLAP = 0x80000000  # bit 31 of a verify result's count: overlapping verify launches
PATH_NONE, PATH_GPU, PATH_CPU = 0, 1, 2  # crc32c_last_path()

PACKET_DTYPE = np.dtype(
    [("payload_off", "<u8"), ("out_idx", "<u8"), ("len", "<u4"), ("bpc", "<u4")], align=True
)
TILE_DTYPE = np.dtype([("src", "<u8"), ("out", "<u4"), ("meta", "<u4")])
GEN_DTYPE = np.dtype([("src", "<u8"), ("out", "<u4"), ("len", "<u4")])
BUFFER_DTYPE = np.dtype([("data", "<u8"), ("len", "<u8")])  # crc32c_buffer (data 0 = zero fill)
FRAME_DTYPE = np.dtype([("frame_off", "<u8"), ("sums_off", "<u8"), ("data_off", "<u8"), ("offset_in_block", "<i8"),
                        ("seqno", "<i8"), ("data_len", "<u4"), ("nsums", "<u4"), ("last", "<u4"),
                        ("reserved", "<u4")])


class FramesResult(ctypes.Structure):
    _fields_ = [("packets", ctypes.c_uint64), ("data_bytes", ctypes.c_uint64), ("checksums", ctypes.c_uint64),
                ("mismatches", ctypes.c_uint64), ("first_bad", ctypes.c_uint64),
                ("first_bad_offset", ctypes.c_int64), ("consumed", ctypes.c_uint64),
                ("last_packet", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class Crc32cError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__("%s (rc=%d %s)" % (msg, rc, errno.errorcode.get(-rc, "?")))
        self.rc = rc


def build(quiet: bool = True) -> str:
    """Compile the library in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    out = subprocess.DEVNULL if quiet else None
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-C", HERE, "-j" + jobs], check=True, stdout=out)
    return LIB_PATH


_LIB = None
_DEBUG_LIB = None


def lib():
    """Load (not build) the shared library; raises if it is missing."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(LIB_PATH + " is not built (run build())")
        # One HIP runtime per process: torch ships its own libamdhip64 and
        # librccl and links them by the unversioned names, so it must be
        # loaded first; our NEEDED libamdhip64.so.7 / librccl.so.1 then bind
        # to the same copies by SONAME.  (Loaded the other way round the
        # process would hold two runtimes and torch would see no device.)
        # torch is plumbing only (device memory, streams, torch.distributed);
        # nothing here computes with it.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _LIB = _bind(ctypes.CDLL(LIB_PATH))
    return _LIB


def debug_lib():
    """libhdfs_crc32c_debug.so (A/B kernel variants, HBM read probe); it links
    against the product library, which is loaded first."""
    global _DEBUG_LIB
    if _DEBUG_LIB is None:
        lib()
        if not os.path.exists(DEBUG_LIB_PATH):
            raise FileNotFoundError(DEBUG_LIB_PATH + " is not built (run build())")
        L = ctypes.CDLL(DEBUG_LIB_PATH)
        vp, i32 = ctypes.c_void_p, ctypes.c_int
        L.crc32c_debug_plan_exec_variant.restype = i32
        L.crc32c_debug_plan_exec_variant.argtypes = [vp, vp, vp, vp, i32, vp]
        L.crc32c_debug_stream_probe.restype = i32
        L.crc32c_debug_stream_probe.argtypes = [vp, ctypes.c_uint64, vp, ctypes.c_uint32, i32, vp]
        L.crc32c_debug_variant_name.restype = ctypes.c_char_p
        L.crc32c_debug_variant_name.argtypes = [i32, ctypes.POINTER(i32)]
        u64p = ctypes.POINTER(ctypes.c_uint64)
        for name, args in (("crc32c_debug_resident_create", [vp, ctypes.c_uint32, ctypes.POINTER(vp)]),
                           ("crc32c_debug_resident_submit", [vp, vp, vp, u64p]),
                           ("crc32c_debug_resident_wait", [vp, ctypes.c_uint64]),
                           ("crc32c_debug_resident_stats", [vp, u64p]),
                           ("crc32c_debug_resident_destroy", [vp])):
            f = getattr(L, name)
            f.restype = i32
            f.argtypes = args
        _DEBUG_LIB = L
    return _DEBUG_LIB


class Resident:
    """crc32c_debug_resident_* (debug library, A/B experiment): a resident
    kernel taking one block's plan over blocks submitted by any thread."""

    def __init__(self, plan: "Plan", idle_us: int = 0):
        h = ctypes.c_void_p()
        L = debug_lib()
        _check(L.crc32c_debug_resident_create(plan.handle, idle_us, ctypes.byref(h)), "crc32c_debug_resident_create")
        self.plan = plan  # (outlives the resident kernel)
        self.handle = h

    def submit(self, dev_payload: int, dev_out: int) -> int:
        t = ctypes.c_uint64(0)
        _check(debug_lib().crc32c_debug_resident_submit(self.handle, ctypes.c_void_p(dev_payload),
                                                        ctypes.c_void_p(dev_out), ctypes.byref(t)),
               "crc32c_debug_resident_submit")
        return int(t.value)

    def wait(self, ticket: int) -> None:
        _check(debug_lib().crc32c_debug_resident_wait(self.handle, ticket), "crc32c_debug_resident_wait")

    def launches(self) -> int:
        n = ctypes.c_uint64(0)
        _check(debug_lib().crc32c_debug_resident_stats(self.handle, ctypes.byref(n)), "crc32c_debug_resident_stats")
        return int(n.value)

    def close(self) -> None:
        if self.handle:
            debug_lib().crc32c_debug_resident_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def variant_info(v: int):
    """(name, exact) of a kernel variant built into the debug library, or None."""
    ex = ctypes.c_int(0)
    name = debug_lib().crc32c_debug_variant_name(v, ctypes.byref(ex))
    return None if name is None else (name.decode(), bool(ex.value))


def _bind(L):
    u32, u64, i32, vp, sz = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t
    pp = ctypes.POINTER(vp)
    sig = {
        "crc32c": (u32, [u32, vp, sz]),
        "crc32c_nchunks": (u64, [u64, u32]),
        "crc32c_packetize": (u64, [u64, u64, u32, u32, vp, u64]),
        "crc32c_batch_nchecksums": (u64, [vp, sz]),
        "crc32c_chunks_cpu": (i32, [vp, sz, u32, vp, u32]),
        "crc32c_device_count": (i32, []),
        "crc32c_ctx_create": (i32, [i32, pp]),
        "crc32c_ctx_destroy": (i32, [vp]),
        "crc32c_plan_create": (i32, [vp, vp, sz, u32, pp]),
        "crc32c_plan_exec": (i32, [vp, vp, vp, vp]),
        "crc32c_plan_destroy": (i32, [vp]),
        "crc32c_plan_nchecksums": (u64, [vp]),
        "crc32c_plan_payload_bytes": (u64, [vp]),
        "crc32c_chunks_dev": (i32, [vp, vp, sz, vp, vp, u32, vp]),
        "crc32c_batch_host": (i32, [vp, vp, vp, sz, vp, u32]),
        "crc32c_chunks": (i32, [vp, sz, u32, vp, u32]),
        "crc32c_multi_create": (i32, [vp, i32, pp]),
        "crc32c_multi_destroy": (i32, [vp]),
        "crc32c_multi_batch_host": (i32, [vp, vp, vp, sz, u32, vp, u32]),
        "crc32c_last_error": (ctypes.c_char_p, []),
        "crc32c_debug_plan": (i32, [vp, sz, vp, sz, vp, sz, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "crc32c_debug_lds_image": (sz, [vp, sz, vp, vp]),
        "crc32c_debug_lds_image_s4": (sz, [vp, sz, u32]),
        "crc32c_plan_verify": (i32, [vp, vp, vp, vp, vp]),
        "crc32c_plan_verify_bitmap": (i32, [vp, vp, vp, vp, vp, vp]),
        "crc32c_frame_packets": (sz, [vp, sz, vp, u32, u64, ctypes.c_int64, u32, vp, sz, vp]),
        "crc32c_block_md5": (None, [vp, sz, u32, vp]),
        "crc32c_verify_host": (ctypes.c_int64, [vp, vp, vp, sz, vp, u32, vp]),
        "crc32c_debug_affine_constants": (None, [u32, vp, vp]),
        "hdfs_crc32": (u32, [u32, vp, sz]),
        "crc32c_last_path": (i32, []),
        "crc32c_plan_create_buffers": (i32, [vp, vp, u32, u64, u64, u64, u32, u32, u32, pp]),
        "crc32c_debug_write_plan": (i32, [vp, u32, u64, u64, u64, u32, u32, vp]),
        "crc32c_multi_unique_id": (i32, [vp]),
        "crc32c_multi_create_rank": (i32, [i32, i32, i32, vp, pp]),
        "crc32c_multi_sync": (i32, [vp]),
        "crc32c_multi_layout": (ctypes.c_int64, [vp, sz, u32, i32, vp, vp]),
        "crc32c_multi_shard_packets": (ctypes.c_int64, [vp, sz, u32, i32, i32, vp, sz]),
        "crc32c_multi_rank_packets": (ctypes.c_int64, [vp, sz, u32, i32, i32, u32, vp, sz]),
        "crc32c_multi_transfers": (ctypes.c_int64, [vp, sz, u32, i32, u32, vp, vp, sz]),
        "crc32c_multi_scatter": (ctypes.c_int64, [vp, sz, u32, i32, u32, vp, vp, sz]),
        "crc32c_multi_plan_create": (i32, [vp, vp, sz, u32, u32, pp]),
        "crc32c_multi_plan_exec": (i32, [vp, vp, vp, vp]),
        "crc32c_multi_plan_join": (i32, [vp, vp]),
        "crc32c_multi_plan_destroy": (i32, [vp]),
        "crc32c_multi_plan_nchecksums": (u64, [vp]),
        "crc32c_multi_plan_shard_bytes": (u64, [vp, i32]),
        "crc32c_multi_plan_gather_ops": (u64, [vp, ctypes.POINTER(ctypes.c_int)]),
        "crc32c_parse_frames": (ctypes.c_int64, [vp, sz, vp, sz, ctypes.POINTER(u64)]),
        "crc32c_plan_exec_blocks": (i32, [vp, vp, vp, sz, vp]),
        "crc32c_blocks_create": (i32, [vp, u32, u32, pp]),
        "crc32c_block_submit": (i32, [vp, vp, vp, ctypes.POINTER(u64)]),
        "crc32c_block_submit_plan": (i32, [vp, vp, vp, vp, ctypes.POINTER(u64)]),
        "crc32c_block_flush": (i32, [vp]),
        "crc32c_block_wait": (i32, [vp, u64]),
        "crc32c_block_checksums": (i32, [vp, vp, vp]),
        "crc32c_blocks_stats": (i32, [vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "crc32c_blocks_destroy": (i32, [vp]),
        "crc32c_blocks_create_resident": (i32, [vp, u32, pp]),
        "crc32c_debug_plan_block": (u64, [vp]),
        "crc32c_debug_blocks_fail_flushes": (i32, [vp, u32]),
        "crc32c_debug_blocks_resident_inject": (i32, [vp, i32, u32]),
        "crc32c_verify_frames_host": (i32, [vp, vp, sz, u32, u64, u32, ctypes.POINTER(FramesResult)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise Crc32cError(rc, "%s: %s" % (what, lib().crc32c_last_error().decode(errors="replace")))


def _np_ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def _stream_handle(stream, keep: dict) -> int:
    """A raw hipStream_t handle from a handle (int, numpy integer, None = the
    default stream) or a stream object (``.cuda_stream``, e.g. a
    ``torch.cuda.Stream``); a stream object is kept alive in ``keep`` (the
    library touches a plan's launch streams until the plan is destroyed)."""
    if stream is None:
        return 0
    if isinstance(stream, numbers.Integral):
        return int(stream)
    h = int(stream.cuda_stream)
    keep.setdefault(h, stream)
    return h


def as_packets(pkts) -> np.ndarray:
    return np.ascontiguousarray(pkts, dtype=PACKET_DTYPE)


# --- 1. drop-in scalar (host CPU, identical to src/crc32c.c:333) ----------
def crc32c(data, crc: int = 0) -> int:
    a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data)
    return int(lib().crc32c(crc & 0xFFFFFFFF, _np_ptr(a), a.nbytes))


def hdfs_crc32(data, crc: int = 0) -> int:
    """Hadoop CHECKSUM_CRC32 on the host (zlib-compatible crc32)."""
    a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data)
    return int(lib().hdfs_crc32(crc & 0xFFFFFFFF, _np_ptr(a), a.nbytes))


def frame_packets(pkts, sums: np.ndarray, flags: int = 0, block_offset: int = 0, first_seqno: int = 0,
                  checksum_len: int = 4):
    """Per-packet send prefixes (PLEN | HLEN | PacketHeaderProto | checksums) of
    a batch: (bytes, offsets[npkts + 1])."""
    pkts = as_packets(pkts)
    sums = np.ascontiguousarray(sums, dtype=np.uint32)
    need = int(lib().crc32c_frame_packets(_np_ptr(pkts), pkts.size, _np_ptr(sums), flags, block_offset,
                                          first_seqno, checksum_len, None, 0, None))
    out = np.zeros(max(need, 1), np.uint8)
    offs = np.zeros(pkts.size + 1, np.uint64)
    got = int(lib().crc32c_frame_packets(_np_ptr(pkts), pkts.size, _np_ptr(sums), flags, block_offset,
                                         first_seqno, checksum_len, _np_ptr(out), out.size, _np_ptr(offs)))
    if got != need:
        raise Crc32cError(-errno.EINVAL, "crc32c_frame_packets")
    return out[:need].tobytes(), offs


def block_md5(sums: np.ndarray, flags: int = 0) -> bytes:
    """OpBlockChecksumResponseProto.md5 of a block's checksums."""
    sums = np.ascontiguousarray(sums, dtype=np.uint32)
    md5 = np.zeros(16, np.uint8)
    lib().crc32c_block_md5(_np_ptr(sums), sums.size, flags, _np_ptr(md5))
    return md5.tobytes()


def nchunks(length: int, bpc: int) -> int:
    return int(lib().crc32c_nchunks(length, bpc))


def packetize(length: int, blockoffset: int, packetsize: int, bpc: int) -> list:
    n = int(lib().crc32c_packetize(length, blockoffset, packetsize, bpc, None, 0))
    lens = np.zeros(max(n, 1), np.uint64)
    lib().crc32c_packetize(length, blockoffset, packetsize, bpc, _np_ptr(lens), n)
    return [int(x) for x in lens[:n]]


def device_count() -> int:
    return int(lib().crc32c_device_count())


# --- 2-4. GPU context, plans, host batches --------------------------------
class Context:
    """One HIP device (crc32c_ctx)."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib().crc32c_ctx_create(device, ctypes.byref(h)), "crc32c_ctx_create")
        self.handle = h
        self.device = device

    def close(self) -> None:
        if self.handle:
            lib().crc32c_ctx_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def plan(self, pkts, flags: int = 0) -> "Plan":
        return Plan(self, pkts, flags)

    def write_plan(self, buffers, bufferoffset: int, length: int, blockoffset: int = 0, packetsize: int = 65536,
                   bpc: int = 512, flags: int = 0) -> "Plan":
        """crc32c_plan_create_buffers: hadoop_rpc_send_packets over a buffer list
        [(device address or 0 for zero fill, length), ...]; exec with payload 0."""
        return Plan(self, None, flags, write=(buffers, bufferoffset, length, blockoffset, packetsize, bpc))

    def verify_frames(self, frames: np.ndarray, bpc: int, chunk_offset: int, flags: int = 0) -> FramesResult:
        """crc32c_verify_frames_host over a buffer of received packet frames."""
        return verify_frames(frames, bpc, chunk_offset, flags, ctx=self)

    def batch_host(self, payload: np.ndarray, pkts, flags: int = 0, out: np.ndarray | None = None) -> np.ndarray:
        """Host-resident batch (crc32c_batch_host): H2D copy -> kernel -> checksums in host memory."""
        pkts = as_packets(pkts)
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        n = total_checksums(pkts)
        if out is None:
            out = np.zeros(max(n, 1), np.uint32)
        _check(lib().crc32c_batch_host(self.handle, _np_ptr(payload), _np_ptr(pkts), pkts.size, _np_ptr(out), flags),
               "crc32c_batch_host")
        return out[:n]

    def verify_host(self, payload: np.ndarray, pkts, expected: np.ndarray, flags: int = 0):
        """Host-resident verification: (number of mismatching checksums, lowest bad index or None)."""
        pkts = as_packets(pkts)
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        expected = np.ascontiguousarray(expected, dtype=np.uint32)
        first = ctypes.c_uint64(0)
        rc = lib().crc32c_verify_host(self.handle, _np_ptr(payload), _np_ptr(pkts), pkts.size, _np_ptr(expected),
                                      flags, ctypes.byref(first))
        if rc < 0:
            _check(int(rc), "crc32c_verify_host")
        return int(rc), (None if first.value == 0xFFFFFFFFFFFFFFFF else int(first.value))

    def chunks_dev(self, pkts, dev_payload: int, dev_out: int, flags: int = 0, stream: int = 0) -> None:
        pkts = as_packets(pkts)
        _check(lib().crc32c_chunks_dev(self.handle, _np_ptr(pkts), pkts.size, ctypes.c_void_p(dev_payload),
                                       ctypes.c_void_p(dev_out), flags, ctypes.c_void_p(stream)), "crc32c_chunks_dev")


class Plan:
    """Device-resident batch plan (crc32c_plan): build once, execute many.

    ``stream`` is a raw HIP stream handle or an object with a ``cuda_stream`` attribute (a
    ``torch.cuda.Stream``). The C library touches every stream a plan ran on when the plan is
    destroyed (include/hdfs_crc32c.h, crc32c_plan_destroy), so a plan must be destroyed before
    its launch streams; a stream object passed here is kept alive by the plan until ``close()``.
    """

    def __init__(self, ctx: Context, pkts, flags: int = 0, write=None):
        h = ctypes.c_void_p()
        if write is None:
            pkts = as_packets(pkts)
            _check(lib().crc32c_plan_create(ctx.handle, _np_ptr(pkts), pkts.size, flags, ctypes.byref(h)),
                   "crc32c_plan_create")
        else:
            buffers, bufferoffset, length, blockoffset, packetsize, bpc = write
            bufs = as_buffers(buffers)
            _check(lib().crc32c_plan_create_buffers(ctx.handle, _np_ptr(bufs), bufs.size, bufferoffset, length,
                                                    blockoffset, packetsize, bpc, flags, ctypes.byref(h)),
                   "crc32c_plan_create_buffers")
        self.ctx = ctx  # keeps the context alive
        self.handle = h
        self._streams = {}  # stream objects launched on, kept alive until close()
        self.nchecksums = int(lib().crc32c_plan_nchecksums(h))
        self.payload_bytes = int(lib().crc32c_plan_payload_bytes(h))

    def _stream(self, stream) -> int:
        return _stream_handle(stream, self._streams)

    def exec(self, dev_payload: int, dev_out: int, stream=0) -> None:
        stream = self._stream(stream)
        _check(lib().crc32c_plan_exec(self.handle, ctypes.c_void_p(dev_payload), ctypes.c_void_p(dev_out),
                                      ctypes.c_void_p(stream)), "crc32c_plan_exec")

    def verify(self, dev_payload: int, dev_expected: int, dev_result: int, stream=0,
               dev_bad_bits: int = 0) -> None:
        """Compare instead of store: dev_result[0] = mismatches, [1] = lowest bad index (async); with
        dev_bad_bits (ceil(nchecksums / 32) u32s) also the bitmap of mismatching checksums
        (crc32c_plan_verify_bitmap)."""
        stream = self._stream(stream)
        if dev_bad_bits:
            _check(lib().crc32c_plan_verify_bitmap(self.handle, ctypes.c_void_p(dev_payload),
                                                   ctypes.c_void_p(dev_expected), ctypes.c_void_p(dev_result),
                                                   ctypes.c_void_p(dev_bad_bits), ctypes.c_void_p(stream)),
                   "crc32c_plan_verify_bitmap")
            return
        _check(lib().crc32c_plan_verify(self.handle, ctypes.c_void_p(dev_payload), ctypes.c_void_p(dev_expected),
                                        ctypes.c_void_p(dev_result), ctypes.c_void_p(stream)), "crc32c_plan_verify")

    def exec_blocks(self, dev_payloads, dev_outs, stream=0) -> None:
        """crc32c_plan_exec_blocks: this plan (one block's shape) on every block, one launch per <= 32."""
        stream = self._stream(stream)
        n = len(dev_payloads)
        pays = (ctypes.c_void_p * max(n, 1))(*[ctypes.c_void_p(x) for x in dev_payloads])
        outs = (ctypes.c_void_p * max(n, 1))(*[ctypes.c_void_p(x) for x in dev_outs])
        _check(lib().crc32c_plan_exec_blocks(self.handle, pays, outs, n, ctypes.c_void_p(stream)),
               "crc32c_plan_exec_blocks")

    def blocks(self, max_blocks: int = 16, window_us: int = 20, resident: bool = False,
               idle_us: int = 0) -> "Blocks":
        """The block queue (crc32c_blocks_create), or its resident-kernel mode
        (crc32c_blocks_create_resident) with ``resident=True``."""
        return Blocks(self, max_blocks, window_us, resident=resident, idle_us=idle_us)

    def exec_variant(self, dev_payload: int, dev_out: int, variant: int, dev_stamps: int = 0, stream: int = 0) -> None:
        """Diagnostic (debug library): run an explicit kernel variant (5/6/36 write per-wave timestamps)."""
        _check(debug_lib().crc32c_debug_plan_exec_variant(self.handle, ctypes.c_void_p(dev_payload),
                                                          ctypes.c_void_p(dev_out), ctypes.c_void_p(dev_stamps),
                                                          variant, ctypes.c_void_p(stream)),
               "crc32c_debug_plan_exec_variant")

    def close(self) -> None:
        if self.handle:
            lib().crc32c_plan_destroy(self.handle)
            self.handle = None
        self._streams = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Blocks:
    """crc32c_blocks: block writes from several threads coalesced into one launch (group commit)."""

    def __init__(self, plan: Plan, max_blocks: int = 16, window_us: int = 20, resident: bool = False,
                 idle_us: int = 0):
        h = ctypes.c_void_p()
        if resident:
            _check(lib().crc32c_blocks_create_resident(plan.handle, idle_us, ctypes.byref(h)),
                   "crc32c_blocks_create_resident")
        else:
            _check(lib().crc32c_blocks_create(plan.handle, max_blocks, window_us, ctypes.byref(h)),
                   "crc32c_blocks_create")
        self.plan = plan  # the plan outlives the queue
        self.handle = h

    def submit(self, dev_payload: int, dev_out: int, plan: "Plan | None" = None) -> int:
        """crc32c_block_submit (plan None: the queue's) / crc32c_block_submit_plan
        (a block of another shape; the plan must outlive its blocks' waits)."""
        t = ctypes.c_uint64(0)
        _check(lib().crc32c_block_submit_plan(self.handle, None if plan is None else plan.handle,
                                              ctypes.c_void_p(dev_payload), ctypes.c_void_p(dev_out),
                                              ctypes.byref(t)), "crc32c_block_submit_plan")
        return int(t.value)

    def flush(self) -> None:
        _check(lib().crc32c_block_flush(self.handle), "crc32c_block_flush")

    def wait(self, ticket: int) -> None:
        _check(lib().crc32c_block_wait(self.handle, ticket), "crc32c_block_wait")

    def checksums(self, dev_payload: int, dev_out: int) -> None:
        """Submit + wait: returns when the block's checksums are in dev_out."""
        _check(lib().crc32c_block_checksums(self.handle, ctypes.c_void_p(dev_payload), ctypes.c_void_p(dev_out)),
               "crc32c_block_checksums")

    def debug_fail_flushes(self, n: int) -> None:
        """crc32c_debug_blocks_fail_flushes: the next n flushes fail at issue (tests of the error path)."""
        _check(lib().crc32c_debug_blocks_fail_flushes(self.handle, n), "crc32c_debug_blocks_fail_flushes")

    def debug_resident_inject(self, hold: bool, fail_waits: int = 0) -> None:
        """crc32c_debug_blocks_resident_inject: hold = no kernel launch (submits queue
        up); the next fail_waits waits return -ETIMEDOUT at once."""
        _check(lib().crc32c_debug_blocks_resident_inject(self.handle, int(hold), fail_waits),
               "crc32c_debug_blocks_resident_inject")

    def stats(self):
        f, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _check(lib().crc32c_blocks_stats(self.handle, ctypes.byref(f), ctypes.byref(b)), "crc32c_blocks_stats")
        return int(f.value), int(b.value)

    def close(self) -> None:
        if self.handle:
            lib().crc32c_blocks_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def multi_unique_id() -> bytes:
    """crc32c_multi_unique_id: the 128-byte RCCL id rank 0 sends to the other ranks."""
    buf = (ctypes.c_uint8 * 128)()
    _check(lib().crc32c_multi_unique_id(buf), "crc32c_multi_unique_id")
    return bytes(buf)


class Multi:
    """Several GPUs of one node (crc32c_multi): all devices of this process
    (``Multi([0, 1, ...])``), or one device of a one-process-per-GPU job
    (``Multi(device=d, rank=r, nranks=n, uid=bytes)``)."""

    def __init__(self, devices=None, device: int = 0, rank: int = 0, nranks: int = 1, uid: bytes | None = None):
        h = ctypes.c_void_p()
        if uid is None:
            devs = (ctypes.c_int * len(devices))(*devices)
            _check(lib().crc32c_multi_create(devs, len(devices), ctypes.byref(h)), "crc32c_multi_create")
            self.local_devices = list(devices)
        else:
            idb = (ctypes.c_uint8 * 128)(*uid)
            _check(lib().crc32c_multi_create_rank(device, rank, nranks, idb, ctypes.byref(h)),
                   "crc32c_multi_create_rank")
            self.local_devices = [device]
        self.handle = h

    def plan(self, pkts, group_packets: int = 64, flags: int = 0) -> "MultiPlan":
        return MultiPlan(self, pkts, group_packets, flags)

    def sync(self) -> None:
        _check(lib().crc32c_multi_sync(self.handle), "crc32c_multi_sync")

    def batch_host(self, payload: np.ndarray, pkts, group_packets: int = 64, flags: int = 0) -> np.ndarray:
        pkts = as_packets(pkts)
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        n = total_checksums(pkts)
        out = np.zeros(max(n, 1), np.uint32)
        _check(lib().crc32c_multi_batch_host(self.handle, _np_ptr(payload), _np_ptr(pkts), pkts.size, group_packets,
                                             _np_ptr(out), flags), "crc32c_multi_batch_host")
        return out[:n]

    def close(self) -> None:
        if self.handle:
            lib().crc32c_multi_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiPlan:
    """Device-resident multi-GPU plan (crc32c_multi_plan): shards + RCCL gather to rank 0."""

    def __init__(self, multi: Multi, pkts, group_packets: int = 64, flags: int = 0):
        pkts = as_packets(pkts)
        h = ctypes.c_void_p()
        _check(lib().crc32c_multi_plan_create(multi.handle, _np_ptr(pkts), pkts.size, group_packets, flags,
                                              ctypes.byref(h)), "crc32c_multi_plan_create")
        self.multi = multi
        self.handle = h
        self._streams = {}  # stream objects launched on, kept alive until close()
        self.nchecksums = int(lib().crc32c_multi_plan_nchecksums(h))

    def shard_bytes(self, rank: int) -> int:
        return int(lib().crc32c_multi_plan_shard_bytes(self.handle, rank))

    def gather_ops(self):
        """crc32c_multi_plan_gather_ops: (point-to-point operations one exec
        posts over the communicator, packed: staging array + scatter kernel)."""
        packed = ctypes.c_int(0)
        n = int(lib().crc32c_multi_plan_gather_ops(self.handle, ctypes.byref(packed)))
        return n, bool(packed.value)

    def exec(self, dev_shards, root_out: int, streams=None) -> None:
        """``streams``: one per local device, handles or stream objects (kept
        alive until close(): the next exec on another stream records an event
        on this one)."""
        n = len(dev_shards)
        shards = (ctypes.c_void_p * n)(*[ctypes.c_void_p(x) for x in dev_shards])
        ss = None if streams is None else (ctypes.c_void_p * n)(
            *[ctypes.c_void_p(_stream_handle(x, self._streams)) for x in streams])
        _check(lib().crc32c_multi_plan_exec(self.handle, shards, ctypes.c_void_p(root_out), ss),
               "crc32c_multi_plan_exec")

    def join(self, streams=None) -> None:
        """crc32c_multi_plan_join (CRC32C_MULTI_PIPELINE plans): every local
        stream waits for every exec issued so far."""
        n = len(self.multi.local_devices)
        ss = None if streams is None else (ctypes.c_void_p * n)(
            *[ctypes.c_void_p(_stream_handle(x, self._streams)) for x in streams])
        _check(lib().crc32c_multi_plan_join(self.handle, ss), "crc32c_multi_plan_join")

    def close(self) -> None:
        if self.handle:
            lib().crc32c_multi_plan_destroy(self.handle)
            self.handle = None
        self._streams = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def multi_layout(pkts, group_packets: int, nranks: int):
    """crc32c_multi_layout: (per-group [rank, shard offset, payload offset, bytes] rows, shard bytes per rank)."""
    pkts = as_packets(pkts)
    n = int(lib().crc32c_multi_layout(_np_ptr(pkts), pkts.size, group_packets, nranks, None, None))
    if n < 0:
        _check(n, "crc32c_multi_layout")
    lay = np.zeros((max(n, 1), 4), np.uint64)
    sb = np.zeros(nranks, np.uint64)
    lib().crc32c_multi_layout(_np_ptr(pkts), pkts.size, group_packets, nranks, _np_ptr(lay), _np_ptr(sb))
    return lay[:n], sb


def multi_shard_packets(pkts, group_packets: int, nranks: int, rank: int) -> np.ndarray:
    """crc32c_multi_shard_packets: rank's packets, payload offsets into its shard, global out indices."""
    pkts = as_packets(pkts)
    n = int(lib().crc32c_multi_shard_packets(_np_ptr(pkts), pkts.size, group_packets, nranks, rank, None, 0))
    if n < 0:
        _check(n, "crc32c_multi_shard_packets")
    out = np.zeros(max(n, 1), PACKET_DTYPE)
    lib().crc32c_multi_shard_packets(_np_ptr(pkts), pkts.size, group_packets, nranks, rank, _np_ptr(out), n)
    return out[:n]


def multi_rank_packets(pkts, group_packets: int, nranks: int, rank: int, flags: int = 0) -> np.ndarray:
    """crc32c_multi_rank_packets: the packets rank's plan computes (payload offsets into its shard, out
    indices into the array it sends to rank 0; rank 0's global unless CRC32C_MULTI_SELF_SEND)."""
    pkts = as_packets(pkts)
    n = int(lib().crc32c_multi_rank_packets(_np_ptr(pkts), pkts.size, group_packets, nranks, rank, flags, None, 0))
    if n < 0:
        _check(n, "crc32c_multi_rank_packets")
    out = np.zeros(max(n, 1), PACKET_DTYPE)
    lib().crc32c_multi_rank_packets(_np_ptr(pkts), pkts.size, group_packets, nranks, rank, flags, _np_ptr(out), n)
    return out[:n]


def multi_transfers(pkts, group_packets: int, nranks: int, flags: int = 0):
    """crc32c_multi_transfers: (local_nout[nranks], transfers[T, 4] = {sending rank, index in its local array,
    file index on rank 0, count}) -- the exchange crc32c_multi_plan_exec posts, in posting order."""
    pkts = as_packets(pkts)
    n = int(lib().crc32c_multi_transfers(_np_ptr(pkts), pkts.size, group_packets, nranks, flags, None, None, 0))
    if n < 0:
        _check(n, "crc32c_multi_transfers")
    ln = np.zeros(nranks, np.uint64)
    xs = np.zeros((max(n, 1), 4), np.uint64)
    lib().crc32c_multi_transfers(_np_ptr(pkts), pkts.size, group_packets, nranks, flags, _np_ptr(ln), _np_ptr(xs), n)
    return ln, xs[:n]


def multi_scatter(pkts, group_packets: int, nranks: int, flags: int = 0):
    """crc32c_multi_scatter: the packed gather's layout -- (stage_off[nranks], tiles[T, 3] = {staging index,
    file index, count}); T = 0 when the gather is not packed (one send / receive per placement)."""
    pkts = as_packets(pkts)
    n = int(lib().crc32c_multi_scatter(_np_ptr(pkts), pkts.size, group_packets, nranks, flags, None, None, 0))
    if n < 0:
        _check(n, "crc32c_multi_scatter")
    so = np.zeros(nranks, np.uint64)
    ts = np.zeros((max(n, 1), 3), np.uint64)
    lib().crc32c_multi_scatter(_np_ptr(pkts), pkts.size, group_packets, nranks, flags, _np_ptr(so), _np_ptr(ts), n)
    return so, ts[:n]


def verify_frames(frames: np.ndarray, bpc: int, chunk_offset: int, flags: int = 0, ctx: Context | None = None):
    """crc32c_verify_frames_host over a buffer of received packet frames; ctx None (no GPU) needs
    CRC32C_CPU_FALLBACK."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    res = FramesResult()
    _check(lib().crc32c_verify_frames_host(None if ctx is None else ctx.handle, _np_ptr(frames), frames.size, bpc,
                                           chunk_offset, flags, ctypes.byref(res)), "crc32c_verify_frames_host")
    return res


def parse_frames(frames: np.ndarray):
    """crc32c_parse_frames: (frame records, bytes consumed)."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    used = ctypes.c_uint64(0)
    n = int(lib().crc32c_parse_frames(_np_ptr(frames), frames.size, None, 0, ctypes.byref(used)))
    if n < 0:
        _check(n, "crc32c_parse_frames")
    info = np.zeros(max(n, 1), FRAME_DTYPE)
    lib().crc32c_parse_frames(_np_ptr(frames), frames.size, _np_ptr(info), n, ctypes.byref(used))
    return info[:n], int(used.value)


def last_path() -> int:
    return int(lib().crc32c_last_path())


def as_buffers(buffers) -> np.ndarray:
    if isinstance(buffers, np.ndarray) and buffers.dtype == BUFFER_DTYPE:
        return np.ascontiguousarray(buffers)
    return np.array([(int(d or 0), int(n)) for d, n in buffers], BUFFER_DTYPE)


def debug_write_plan(buffers, bufferoffset: int, length: int, blockoffset: int = 0, packetsize: int = 65536,
                     bpc: int = 512) -> dict:
    bufs = as_buffers(buffers)
    c = np.zeros(6, np.uint64)
    _check(lib().crc32c_debug_write_plan(_np_ptr(bufs), bufs.size, bufferoffset, length, blockoffset, packetsize,
                                         bpc, _np_ptr(c)), "crc32c_debug_write_plan")
    return dict(zip(["tiles", "gen", "seg", "pieces", "consts", "nchecksums"], (int(x) for x in c)))


def chunks_cpu(packet: np.ndarray, bpc: int, flags: int = 0) -> np.ndarray:
    """The reference's per-packet loop on one host packet, on the host CPU."""
    packet = np.ascontiguousarray(packet, dtype=np.uint8)
    n = nchunks(packet.size, bpc)
    out = np.zeros(max(n, 1), np.uint32)
    _check(lib().crc32c_chunks_cpu(_np_ptr(packet), packet.size, bpc, _np_ptr(out), flags), "crc32c_chunks_cpu")
    return out[:n]


def batch_host_cpu(payload: np.ndarray, pkts, flags: int = 0, out: np.ndarray | None = None) -> np.ndarray:
    """The product's host-CPU path over a host batch (crc32c_batch_host with no GPU context and
    CRC32C_CPU_FALLBACK: crc32c_chunks_cpu per packet on the calling thread)."""
    pkts = as_packets(pkts)
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    n = total_checksums(pkts)
    if out is None:
        out = np.zeros(max(n, 1), np.uint32)
    _check(lib().crc32c_batch_host(None, _np_ptr(payload), _np_ptr(pkts), pkts.size, _np_ptr(out),
                                   flags | CRC32C_CPU_FALLBACK), "crc32c_batch_host (CPU)")
    return out[:n]


def chunks(packet: np.ndarray, bpc: int, flags: int = 0) -> np.ndarray:
    """The reference's per-packet loop on one host packet, on the default GPU context."""
    packet = np.ascontiguousarray(packet, dtype=np.uint8)
    n = nchunks(packet.size, bpc)
    out = np.zeros(max(n, 1), np.uint32)
    _check(lib().crc32c_chunks(_np_ptr(packet), packet.size, bpc, _np_ptr(out), flags), "crc32c_chunks")
    return out[:n]


# --- helpers ----------------------------------------------------------------
def total_checksums(pkts) -> int:
    pkts = as_packets(pkts)
    return int(lib().crc32c_batch_nchecksums(_np_ptr(pkts), pkts.size))


def debug_plan(pkts):
    """Work items a plan would upload (FastTile / GenItem arrays)."""
    pkts = as_packets(pkts)
    nt, ng = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().crc32c_debug_plan(_np_ptr(pkts), pkts.size, None, 0, None, 0, ctypes.byref(nt), ctypes.byref(ng)),
           "crc32c_debug_plan")
    tiles = np.zeros(max(nt.value, 1), TILE_DTYPE)
    gen = np.zeros(max(ng.value, 1), GEN_DTYPE)
    _check(lib().crc32c_debug_plan(_np_ptr(pkts), pkts.size, _np_ptr(tiles), nt.value, _np_ptr(gen), ng.value,
                                   ctypes.byref(nt), ctypes.byref(ng)), "crc32c_debug_plan")
    return tiles[: nt.value], gen[: ng.value]


def debug_lds_image():
    """The kernel's LDS image and affine constants (c_lg[5], c_small[4])."""
    n = int(lib().crc32c_debug_lds_image(None, 0, None, None))
    img = np.zeros(n, np.uint8)
    c_lg = np.zeros(5, np.uint32)
    c_small = np.zeros(4, np.uint32)
    lib().crc32c_debug_lds_image(_np_ptr(img), n, _np_ptr(c_lg), _np_ptr(c_small))
    return img, c_lg, c_small


def debug_lds_image_s4(flags: int = 0):
    """The slicing-by-4 kernel's LDS image (CRC32C, or CRC32 with CRC32C_TYPE_CRC32)."""
    n = int(lib().crc32c_debug_lds_image_s4(None, 0, flags))
    img = np.zeros(n, np.uint8)
    lib().crc32c_debug_lds_image_s4(_np_ptr(img), n, flags)
    return img


def debug_affine_constants(flags: int = 0):
    c_lg = np.zeros(5, np.uint32)
    c_small = np.zeros(4, np.uint32)
    lib().crc32c_debug_affine_constants(flags, _np_ptr(c_lg), _np_ptr(c_small))
    return c_lg, c_small
