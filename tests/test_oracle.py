"""The oracle is pinned before it is trusted: every published vector, every
fixture generated from the reference itself, and (where it is built) the
reference's own code run side by side."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import oracle
from conftest import golden_batch_packets, golden_fill


def test_published_known_answers(orc, golden):
    for e in golden["known_answers"]["published"]:
        data = bytes.fromhex(e["hex"])
        assert "%08x" % orc.crc32c(data) == e["crc"], e["name"]
        assert "%08x" % orc.crc32c(data, bytewise=True) == e["crc"], e["name"]
        assert "%08x" % oracle.py_crc32c(data) == e["crc"], e["name"]


def test_derived_known_answers(orc, golden):
    for e in golden["known_answers"]["derived"]:
        data = golden_fill(e["kind"], e["len"], 0)
        assert "%08x" % orc.crc32c(data) == e["crc"], e["name"]
    zeros512 = [e for e in golden["known_answers"]["derived"] if e["name"] == "zeros_512"][0]
    assert zeros512["crc"] == "30fcedc0"


def test_chained_crc_argument(orc, golden):
    for e in golden["known_answers"]["chained"]:
        buf = golden_fill("xorshift", e["len"], e["seed"])
        first = orc.crc32c(buf[: e["split"]])
        assert "%08x" % first == e["first"]
        assert "%08x" % orc.crc32c(buf[e["split"]:], first) == e["crc"]
        assert "%08x" % orc.crc32c(buf) == e["oneshot"]


def test_reference_stdin_harness_values(orc, golden):
    # crc32c.c:345-382 chains 786432-byte slices through the crc argument.
    for e in golden["known_answers"]["stdin_harness"]:
        buf = golden_fill("xorshift", e["len"], e["seed"])
        crc = 0
        for off in range(0, buf.size, 786432):
            crc = orc.crc32c(buf[off:off + 786432], crc)
        assert "%08x" % crc == e["crc"]


def test_packet_fixtures(orc, golden):
    for c in golden["packets"]["cases"]:
        buf = golden_fill(c["kind"], c["len"] + c["skip"], c["seed"])[c["skip"]:]
        got = orc.chunks(buf, c["bpc"])
        assert ["%08x" % v for v in got] == c["crcs"], (c["bpc"], c["kind"], c["len"])


@pytest.mark.parametrize("name", ["c1_one_packet", "c3_one_block_4MiB", "c5_mixed_bpc_96", "ragged_tail_257"])
def test_batch_digests(orc, golden, name):
    spec = [b for b in golden["batches"] if b["name"] == name][0]
    pk = golden_batch_packets(spec)
    payload = oracle.xorshift64_bytes(spec["payload_bytes"], spec["seed"])
    got = orc.batch(payload, pk, spec["nchecksums"])
    assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == spec["sha256_le"]
    assert ["%08x" % v for v in got[:8]] == spec["head"]


def test_big_endian_is_htonl(orc):
    buf = oracle.xorshift64_bytes(5000, 3)
    le = orc.chunks(buf, 512)
    be = orc.chunks(buf, 512, big_endian=True)
    assert np.array_equal(be, le.byteswap())


def test_bytewise_equals_slice8_unaligned(orc):
    rng = np.random.default_rng(5)
    buf = oracle.xorshift64_bytes(70000, 9)
    for _ in range(200):
        off = int(rng.integers(0, 64))
        n = int(rng.integers(0, 3000))
        crc = int(rng.integers(0, 2**32))
        seg = buf[off:off + n]
        assert orc.crc32c(seg, crc) == orc.crc32c(seg, crc, bytewise=True)


def test_python_restatement_small(orc):
    buf = oracle.xorshift64_bytes(300, 17)
    for n in (0, 1, 5, 64, 299):
        assert oracle.py_crc32c(buf[:n].tobytes()) == orc.crc32c(buf[:n])


def test_packetize_hand_examples(orc):
    # hadooprpc.c:827-857 worked by hand: full 64 KiB packets then the empty
    # end-of-block packet; a block offset off the chunk grid first finishes
    # that chunk (832-840).
    assert orc.packetize(131072, 0, 65536, 512) == [65536, 65536, 0]
    assert orc.packetize(1000, 0, 65536, 512) == [1000, 0]
    assert orc.packetize(70000, 100, 65536, 512) == [412, 65536, 70000 - 412 - 65536, 0]
    assert orc.packetize(0, 0, 65536, 512) == [0]
    # trim clamped to the bytes left (the reference only asserts, hadooprpc.c:622)
    assert orc.packetize(50, 10, 65536, 512) == [50, 0]


@pytest.mark.skipif(not oracle.Reference.available(), reason="reference build not present")
def test_oracle_matches_reference_random(orc):
    ref = oracle.Reference()
    rng = np.random.default_rng(11)
    buf = oracle.xorshift64_bytes(1 << 17, 21)
    for _ in range(500):
        off = int(rng.integers(0, 4096))
        n = int(rng.integers(0, 9000))
        crc = int(rng.integers(0, 2**32))
        assert ref.crc32c(buf[off:off + n], crc) == orc.crc32c(buf[off:off + n], crc)
    pk = oracle.mixed_packets(12, pkt_len=20000, bpcs=(512, 100, 4096, 1536))
    payload = oracle.xorshift64_bytes(12 * 20000, 4)
    n = oracle.total_checksums(pk)
    assert np.array_equal(ref.batch(payload, pk, n), orc.batch(payload, pk, n))
