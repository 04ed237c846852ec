"""The C caller of INTEGRATION.md section 3 (examples/block_write.c, built by
native-hdfs-fuse_amd/Makefile against include/hdfs_crc32c.h): a block write
cut by crc32c_packetize, checksummed in one crc32c_batch_host call, framed by
crc32c_frame_packets and verified by crc32c_verify_host, each step checked
inside the program against the reference's per-chunk loop (hadooprpc.c:
733-742) done with the drop-in crc32c().  Run as a child process."""
from __future__ import annotations

import os
import subprocess

import pytest

from conftest import ROOT

EXE = os.path.join(ROOT, "examples", "block_write")

# (len, blockoffset, bpc): a 4 MiB block; a write starting off a chunk
# boundary (trimmed first packet, hadooprpc.c:832-840); bpc 4096 and 1024
# with a short tail; a write smaller than one chunk; an empty write.
CASES = [(4 << 20, 0, 512), (1_000_000, 1234, 512), (3 * 65536 + 77, 100, 4096), (700_001, 0, 1024),
         (300, 5, 512), (0, 0, 512)]


def _run(args, timeout):
    if not os.path.exists(EXE):
        pytest.fail(EXE + " is not built (run __graft_entry__.build())")
    r = subprocess.run([EXE] + [str(a) for a in args], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok:"), r.stdout
    return r.stdout


@pytest.mark.parametrize("length,blockoffset,bpc", CASES)
def test_c_caller_cpu_side(length, blockoffset, bpc):
    """No GPU: packetize, scalar crc32c and framing exact; the GPU entry
    points fail with -ENODEV instead of computing on the CPU."""
    if os.environ.get("HIP_VISIBLE_DEVICES") is None and os.path.exists("/dev/kfd"):
        pytest.skip("a GPU may be visible here; the GPU test covers this path")
    _run(["--cpu", length, blockoffset, bpc], 60)


@pytest.mark.gpu
@pytest.mark.parametrize("length,blockoffset,bpc", CASES)
def test_c_caller_gpu(length, blockoffset, bpc):
    """Through the GPU: every checksum of the block equals crc32c() per chunk,
    the framed prefixes carry them, verification finds 0 and then exactly
    the one flipped checksum."""
    _run([length, blockoffset, bpc], 120)


FUSE_EXE = os.path.join(ROOT, "examples", "fuse_write")
# (TRUNCATE, NULLPADDING, THEDATA, TRAILINGDATA lengths, blockoffset, bpc):
# hadoop_fuse_write's four buffers (fuse.c:1348-1354) in the shapes a write
# into an existing block, a write past EOF, a plain block write and a small
# random write produce; packet cutting from a block offset off a chunk
# boundary; bpc 1536.
FUSE_CASES = [(10000, 300000, 1 << 20, 77777, 0, 512), (0, 0, 4 << 20, 0, 0, 512),
              (5000, 20000, 200000, 3000, 1037, 512), (12345, 0, 100000, 0, 1536 * 3, 1536),
              (3, 1, 700, 5, 0, 512), (0, 4096, 0, 0, 0, 512)]


@pytest.mark.gpu
@pytest.mark.parametrize("case", FUSE_CASES)
def test_c_caller_fuse_write_buffers(case):
    """examples/fuse_write.c: the FUSE write path from C with the buffers in
    device memory -- crc32c_plan_create_buffers / exec / verify_bitmap --
    exact against crc32c() per chunk over the host-assembled stream, the
    bitmap naming exactly the flipped checksums, and an all-NULL ftruncate
    extension giving the zero-chunk constant."""
    if not os.path.exists(FUSE_EXE):
        pytest.fail(FUSE_EXE + " is not built (run __graft_entry__.build())")
    r = subprocess.run([FUSE_EXE] + [str(a) for a in case], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok:"), r.stdout
