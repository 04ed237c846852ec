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


def test_verify_frames_without_gpu_cpu_fallback():
    """crc32c_verify_frames_host with ctx = NULL (no usable GPU) and
    CRC32C_CPU_FALLBACK verifies on the host CPU (the product's
    crc32c_chunks_cpu); without the flag it is refused.  Malformed or
    misplaced frames fail with -EBADMSG and say why in crc32c_last_error()."""
    hdfs = load_package()
    bpc, chunk_offset = 512, 3 * 512
    pk = _block_packets(hdfs, 300000, chunk_offset, bpc)
    payload = oracle.xorshift64_bytes(300000 + 16, 5)
    sums = oracle.Oracle().batch(payload, pk, hdfs.total_checksums(pk))
    pre, offs = hdfs.frame_packets(pk, sums, 0, block_offset=chunk_offset)
    parts = []
    for i in range(pk.size):
        parts.append(np.frombuffer(pre[int(offs[i]):int(offs[i + 1])], np.uint8))
        parts.append(payload[int(pk["payload_off"][i]):int(pk["payload_off"][i]) + int(pk["len"][i])])
    fr = np.concatenate(parts)
    r = hdfs.verify_frames(fr, bpc, chunk_offset, hdfs.CRC32C_CPU_FALLBACK)
    assert (r.packets, r.mismatches, r.first_bad, r.checksums, r.last_packet) == (
        pk.size, 0, 2**64 - 1, hdfs.total_checksums(pk), 1)
    assert hdfs.last_path() == hdfs.PATH_CPU
    info, _ = hdfs.parse_frames(fr)
    bad = fr.copy()
    bad[int(info["data_off"][2]) + 3 * bpc + 1] ^= 4
    r = hdfs.verify_frames(bad, bpc, chunk_offset, hdfs.CRC32C_CPU_FALLBACK)
    assert (r.mismatches, r.first_bad) == (1, hdfs.total_checksums(pk[:2]) + 3)
    assert r.first_bad_offset == chunk_offset + int(pk["payload_off"][2]) + 3 * bpc
    with pytest.raises(hdfs.Crc32cError) as e:
        hdfs.verify_frames(fr, bpc, chunk_offset)  # no GPU, no fallback
    assert e.value.rc == -22
    with pytest.raises(hdfs.Crc32cError) as e:
        hdfs.verify_frames(fr, bpc, chunk_offset + bpc, hdfs.CRC32C_CPU_FALLBACK)
    assert e.value.rc == -74 and "offsetInBlock" in str(e.value)
    trunc = fr.copy()
    trunc[:4] = np.frombuffer(struct.pack(">I", 3), np.uint8)  # PLEN < 4
    with pytest.raises(hdfs.Crc32cError) as e:
        hdfs.parse_frames(trunc)
    assert e.value.rc == -74 and "PLEN" in str(e.value)
