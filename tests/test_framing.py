"""Host-side companions of the checksum path (SURVEY.md section 8f rows 2
and 4): batched packet framing and the block MD5-of-CRCs.  Oracles: Google's
protobuf runtime encoding PacketHeaderProto from its datatransfer.proto
definition (datatransfer.proto:184-191, rebuilt here as a descriptor -- no
protoc in this image), Python's struct for PLEN / HLEN, hashlib's MD5."""
from __future__ import annotations

import hashlib
import struct

import numpy as np
import pytest

import oracle
from conftest import load_package


@pytest.fixture(scope="module")
def header_cls():
    pb = pytest.importorskip("google.protobuf")
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    assert pb is not None
    fdp = descriptor_pb2.FileDescriptorProto(name="datatransfer_min.proto", package="hadoop.hdfs", syntax="proto2")
    m = fdp.message_type.add(name="PacketHeaderProto")
    F = descriptor_pb2.FieldDescriptorProto
    for name, num, ty, lab in [("offsetInBlock", 1, F.TYPE_SFIXED64, F.LABEL_REQUIRED),
                               ("seqno", 2, F.TYPE_SFIXED64, F.LABEL_REQUIRED),
                               ("lastPacketInBlock", 3, F.TYPE_BOOL, F.LABEL_REQUIRED),
                               ("dataLen", 4, F.TYPE_SFIXED32, F.LABEL_REQUIRED),
                               ("syncBlock", 5, F.TYPE_BOOL, F.LABEL_OPTIONAL)]:
        m.field.add(name=name, number=num, type=ty, label=lab)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("hadoop.hdfs.PacketHeaderProto"))


def _block_packets(hdfs, length, blockoffset, bpc, packetsize=65536):
    lens = hdfs.packetize(length, blockoffset, packetsize, bpc)
    pk = np.zeros(len(lens), hdfs.PACKET_DTYPE)
    pk["len"] = lens
    pk["bpc"] = bpc
    pk["payload_off"] = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    per = (pk["len"].astype(np.uint64) + bpc - 1) // bpc
    pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    return pk


@pytest.mark.parametrize("length,blockoffset,bpc", [(4 << 20, 0, 512), (200000, 700, 512), (70000, 0, 4096),
                                                    (0, 0, 512), (513, 511, 512)])
def test_frame_packets_matches_reference_wire_format(header_cls, length, blockoffset, bpc):
    hdfs = load_package()
    pk = _block_packets(hdfs, length, blockoffset, bpc)
    payload = oracle.xorshift64_bytes(max(length, 1), 9)
    sums = oracle.Oracle().batch(payload, pk, hdfs.total_checksums(pk))
    for flags, s in ((0, sums), (hdfs.CRC32C_BIG_ENDIAN, sums.byteswap())):
        buf, offs = hdfs.frame_packets(pk, s, flags, block_offset=blockoffset, first_seqno=0)
        want = b""
        for i, p in enumerate(pk):
            n = (int(p["len"]) + bpc - 1) // bpc
            hdr = header_cls(offsetInBlock=blockoffset + int(p["payload_off"]), seqno=i,
                             lastPacketInBlock=int(p["len"]) == 0, dataLen=int(p["len"])).SerializeToString()
            pre = struct.pack(">IH", 4 + 4 * n + int(p["len"]), len(hdr)) + hdr
            pre += struct.pack(">%dI" % n, *[int(x) for x in sums[int(p["out_idx"]):int(p["out_idx"]) + n]])
            assert int(offs[i]) == len(want)
            want += pre
        assert buf == want
        assert int(offs[-1]) == len(want)
    # the reference ends every block with an empty packet (hadooprpc.c:853-856)
    assert int(pk["len"][-1]) == 0


def test_frame_packets_checksum_null_and_small_buffer(header_cls):
    hdfs = load_package()
    pk = _block_packets(hdfs, 100000, 0, 512)
    buf, offs = hdfs.frame_packets(pk, np.zeros(1, np.uint32), checksum_len=0)
    assert len(buf) == pk.size * (6 + 25)
    L = hdfs.lib()
    import ctypes
    need = L.crc32c_frame_packets(pk.ctypes.data_as(ctypes.c_void_p), pk.size, None, 0, 0, 0, 0, None, 0, None)
    assert need == len(buf)
    assert L.crc32c_frame_packets(pk.ctypes.data_as(ctypes.c_void_p), pk.size, None, 0, 0, 0, 3, None, 0, None) == 0


def test_block_md5_of_crcs():
    hdfs = load_package()
    pk = oracle.uniform_packets(64)  # one 4 MiB block
    payload = oracle.xorshift64_bytes(64 * 65536, 21)
    sums = oracle.Oracle().batch(payload, pk, hdfs.total_checksums(pk))
    want = hashlib.md5(sums.astype(">u4").tobytes()).digest()
    assert hdfs.block_md5(sums) == want
    assert hdfs.block_md5(sums.byteswap(), hdfs.CRC32C_BIG_ENDIAN) == want
    for n in (0, 1, 13, 255, 256, 257, 1000):
        assert hdfs.block_md5(sums[:n]) == hashlib.md5(sums[:n].astype(">u4").tobytes()).digest(), n
