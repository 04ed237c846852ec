"""CPU checks of libhdfs_crc32c.so: it loads, exports every symbol the headers
declare, its drop-in scalar crc32c() and packet helpers match the oracle, its
work decomposition covers every chunk exactly once, and a bit-level model of
the kernel evaluated on the library's own LDS image reproduces the oracle."""
from __future__ import annotations

import glob
import os
import re

import numpy as np
import pytest

import oracle
from conftest import ROOT, golden_fill
from kernel_model import KernelModel, KernelModelS4


def _declared_functions(debug_only: bool = False):
    """crc32c* functions the headers declare: the product library's, or
    (debug_only) section 2 of hdfs_crc32c_debug.h, which only
    libhdfs_crc32c_debug.so exports."""
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        if h.endswith("_debug.h"):
            head, _, tail = text.partition("/* ---- 2. libhdfs_crc32c_debug.so only ---- */")
            text = tail if debug_only else head
        elif debug_only:
            continue
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(crc32c\w*)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return names


def test_exports_every_declared_symbol(hdfs):
    names = _declared_functions()
    assert "crc32c" in names and "crc32c_plan_exec" in names and len(names) >= 20
    lib = hdfs.lib()
    for n in sorted(names):
        assert hasattr(lib, n), n
    dbg = _declared_functions(debug_only=True)
    assert dbg == {"crc32c_debug_plan_exec_variant", "crc32c_debug_variant_name", "crc32c_debug_stream_probe",
                   "crc32c_debug_resident_create", "crc32c_debug_resident_submit", "crc32c_debug_resident_wait",
                   "crc32c_debug_resident_stats", "crc32c_debug_resident_trace", "crc32c_debug_resident_destroy"}
    dlib = hdfs.debug_lib()
    for n in sorted(dbg):
        assert hasattr(dlib, n), n


def test_product_library_has_no_variant_switch(hdfs):
    """The public path launches only the production kernel: the product .so
    exports no variant entry point or read probe, never reads a kernel-variant
    environment variable, and holds exactly the twenty-two production
    kernels (exec, verify; full image without general-tile code, with
    general tiles and shifted tiles, general tiles only, shifted tiles only;
    compact image, compact image with quarter units, with quarter units and
    early loads, with half units, and the aligned one-block form -- quarter
    units, early loads, no general-tile code, 8 waves; half tiles with
    general tiles, with and without shifted tiles); the A/B kernels live in
    the debug library."""
    import ctypes

    lib = ctypes.CDLL(hdfs.LIB_PATH)
    for n in _declared_functions(debug_only=True):
        assert not hasattr(lib, n), n
    blob = open(hdfs.LIB_PATH, "rb").read()
    assert b"KVARIANT" not in blob
    kernels = set(re.findall(rb"_Z23hdfs_crc32c_plan_kernelILi\d+ELi\d+ELi\d+EEvN8hdfs_crc7KParamsE", blob))
    # modes: 3 = S4 | NT, + 64 verify, + 256 general-tile code, + 512 compact image (small batches),
    # + 4096 quarter units (the smallest batches), + 32768 no shifted tiles, + 65536 no general tiles,
    # + 131072 general items' next subtile facts hoisted (the build with both general and shifted tiles),
    # + 1048576 half tiles (their own builds: general tiles, with and without shifted tiles),
    # + 2097152 (NP) no padded power-of-two tiles (the small-batch builds),
    # + 1024 first unit's loads before the staging, + 16384 half units (2 per tile)
    NP = 2097152
    want = {b"_Z23hdfs_crc32c_plan_kernelILi768ELi3ELi%dEEvN8hdfs_crc7KParamsE" % m
            for m in (3, 67, 131331, 131395, 771 + NP, 835 + NP, 4867 + NP, 4931 + NP, 5891 + NP, 5955 + NP,
                      21251 + NP, 21315 + NP, 33027, 33091, 65795, 65859, 1081603, 1081667, 1179907, 1179971)}
    want |= {b"_Z23hdfs_crc32c_plan_kernelILi512ELi2ELi%dEEvN8hdfs_crc7KParamsE" % m for m in (5635, 5699)}
    assert kernels == want, kernels
    dblob = open(hdfs.DEBUG_LIB_PATH, "rb").read()
    assert len(set(re.findall(rb"_Z23hdfs_crc32c_plan_kernelILi\d+ELi\d+ELi\d+EEvN8hdfs_crc7KParamsE", dblob))) >= 9


def test_product_library_does_not_use_the_oracle(hdfs):
    """The checker never ships: the product library (and the debug library
    built beside it) neither links nor names anything under oracle/ -- no
    oracle / reference-harness symbol, no oracle library in NEEDED."""
    import subprocess

    for path in (hdfs.LIB_PATH, hdfs.DEBUG_LIB_PATH):
        blob = open(path, "rb").read()
        for marker in (b"oracle_batch", b"oracle_crc32c", b"ref_batch", b"liboracle", b"crc32c_oracle", b"oracle/_ref"):
            assert marker not in blob, (path, marker)
        needed = subprocess.run(["readelf", "-d", path], capture_output=True, text=True).stdout
        assert "oracle" not in needed and "_ref" not in needed, needed


def test_scalar_dropin_known_answers(hdfs, golden):
    for e in golden["known_answers"]["published"]:
        assert "%08x" % hdfs.crc32c(bytes.fromhex(e["hex"])) == e["crc"]
    for e in golden["known_answers"]["derived"]:
        assert "%08x" % hdfs.crc32c(golden_fill(e["kind"], e["len"], 0)) == e["crc"], e["name"]
    for e in golden["known_answers"]["chained"]:
        buf = golden_fill("xorshift", e["len"], e["seed"])
        c1 = hdfs.crc32c(buf[: e["split"]])
        assert "%08x" % hdfs.crc32c(buf[e["split"]:], c1) == e["crc"]


def test_scalar_dropin_random_vs_oracle(hdfs, orc):
    # sizes around the three-stripe groups (3 x 168 / 336 / 1024 / 8192 bytes)
    # and their cascades, with unaligned starts
    rng = np.random.default_rng(1)
    buf = oracle.xorshift64_bytes(1 << 17, 33)
    for n in list(range(0, 40)) + [503, 504, 505, 511, 512, 513, 1007, 1008, 1009, 1024, 1512, 3071, 3072, 3073,
                                   4096, 6144, 9999, 24575, 24576, 24577, 65000, 65536, 100000]:
        off = int(rng.integers(0, 16))
        crc = int(rng.integers(0, 2**32))
        seg = buf[off:off + n]
        assert hdfs.crc32c(seg, crc) == orc.crc32c(seg, crc), n


@pytest.mark.skipif(not oracle.Reference.available(), reason="reference build not present")
def test_scalar_dropin_matches_reference_build(hdfs):
    """The drop-in against the reference's own crc32c.c (oracle/_ref): random
    lengths across every stripe size, random alignment and incoming crc."""
    ref = oracle.Reference()
    rng = np.random.default_rng(77)
    buf = oracle.xorshift64_bytes(1 << 17, 78)
    for _ in range(400):
        off = int(rng.integers(0, 64))
        n = int(rng.choice([int(rng.integers(0, 2048)), int(rng.integers(2048, 70000))]))
        crc = int(rng.integers(0, 2**32))
        seg = buf[off:off + n]
        assert hdfs.crc32c(seg, crc) == ref.crc32c(seg, crc), (off, n)


def test_nchunks_and_packetize(hdfs, orc):
    assert hdfs.nchunks(65536, 512) == 128
    assert hdfs.nchunks(65537, 512) == 129
    assert hdfs.nchunks(0, 512) == 0
    for args in [(131072, 0, 65536, 512), (70000, 100, 65536, 512), (4194304, 0, 65536, 512),
                 (1000, 513, 65536, 1024), (50, 10, 65536, 512), (0, 0, 65536, 512), (10**6, 12345, 65536, 4096)]:
        assert hdfs.packetize(*args) == orc.packetize(*args), args


def test_zero_length_and_zero_bpc_packets_agree(hdfs):
    """One rule across the ABI: a zero-length packet (the block's final empty
    packet, hadooprpc.c:853-856) has no checksums whatever its bpc -- it is
    counted by nothing and accepted by the plan builder; a packet with data
    and bpc == 0 is refused by the plan builder and counts nothing."""
    pk = oracle.uniform_packets(3, 65536, 512)
    end = np.zeros(1, pk.dtype)  # len 0, bpc 0: as the reference's last packet could be written
    end["payload_off"] = 3 * 65536
    for tail_bpc in (0, 512):
        end["bpc"] = tail_bpc
        b = np.concatenate([pk, end])
        assert hdfs.total_checksums(b) == oracle.total_checksums(b) == 3 * 128
        tiles, gen = hdfs.debug_plan(b)
        assert tiles.size == 3 * 8 and gen.size == 0
    bad = pk.copy()
    bad["bpc"][1] = 0
    assert hdfs.total_checksums(bad) == 3 * 128  # packet 1 counts nothing; packet 2 ends at 384
    with pytest.raises(hdfs.Crc32cError):
        hdfs.debug_plan(bad)


def test_chunks_cpu_matches_reference_loop(hdfs, orc, golden):
    """crc32c_chunks_cpu (the per-packet loop of hadooprpc.c:733-742 on the
    host, whole chunks as 3 interleaved crc32q chains): every golden packet
    vector, random packets of every bpc shape against the oracle, wire
    order, CHECKSUM_CRC32 against zlib, and argument errors."""
    import zlib

    for c in golden["packets"]["cases"]:
        buf = golden_fill(c["kind"], c["len"] + c["skip"], c["seed"])[c["skip"]:]
        got = hdfs.chunks_cpu(np.ascontiguousarray(buf), c["bpc"])
        assert ["%08x" % v for v in got] == c["crcs"], (c["bpc"], c["kind"], c["len"])
    rng = np.random.default_rng(23)
    data = oracle.xorshift64_bytes(300_000, 23)
    for _ in range(60):
        bpc = int(rng.choice([512, 1024, 4096, 8, 24, 100, 1536, 7, 65536]))
        off, n = int(rng.integers(0, 64)), int(rng.integers(0, 200_000))
        pkt = np.ascontiguousarray(data[off:off + n])
        want = orc.chunks(pkt, bpc)
        assert np.array_equal(hdfs.chunks_cpu(pkt, bpc), want), (bpc, off, n)
        assert np.array_equal(hdfs.chunks_cpu(pkt, bpc, hdfs.CRC32C_BIG_ENDIAN), want.byteswap())
        ieee = [zlib.crc32(pkt[i:i + bpc].tobytes()) for i in range(0, n, bpc)]
        assert hdfs.chunks_cpu(pkt, bpc, hdfs.CRC32C_TYPE_CRC32).tolist() == ieee
    L = hdfs.lib()
    out = np.zeros(4, np.uint32)
    assert L.crc32c_chunks_cpu(data.ctypes.data, 100, 0, out.ctypes.data, 0) == -22
    assert L.crc32c_chunks_cpu(data.ctypes.data, 100, 512, out.ctypes.data, 0x80) == -22
    assert L.crc32c_chunks_cpu(None, 0, 512, None, 0) == 0


@pytest.mark.parametrize("name", ["c1_one_packet", "c3_one_block_4MiB", "c5_mixed_bpc_96", "ragged_tail_257"])
def test_chunks_cpu_golden_batches(hdfs, golden, name):
    """BASELINE config 1 (one 64 KiB packet, the CPU path) and the other small
    golden batches through crc32c_chunks_cpu packet by packet: SHA-256 of the
    checksum array equals the reference build's (tests/golden/batches.json)."""
    import hashlib

    spec = [b for b in golden["batches"] if b["name"] == name][0]
    from conftest import golden_batch_packets

    pk = golden_batch_packets(spec)
    payload = oracle.xorshift64_bytes(spec["payload_bytes"], spec["seed"])
    out = np.zeros(spec["nchecksums"], np.uint32)
    for p in pk:
        off, idx, ln, bpc = int(p["payload_off"]), int(p["out_idx"]), int(p["len"]), int(p["bpc"])
        n = hdfs.nchunks(ln, bpc)
        out[idx:idx + n] = hdfs.chunks_cpu(np.ascontiguousarray(payload[off:off + ln]), bpc)
    assert hashlib.sha256(out.astype("<u4").tobytes()).hexdigest() == spec["sha256_le"]


def test_batch_nchecksums(hdfs):
    """crc32c_batch_nchecksums (the checksum array length of a batch): the
    oracle's count on full batches; with empty packets (which own no
    checksum) and reversed out_idx, the max end over non-empty packets."""
    rng = np.random.default_rng(17)
    assert hdfs.total_checksums(np.zeros(0, oracle.PACKET_DTYPE)) == 0
    for pk in [oracle.uniform_packets(4096), oracle.mixed_packets(96), next(c for n, c in _cases() if n == "odd")]:
        assert hdfs.total_checksums(pk) == oracle.total_checksums(pk)
    for _ in range(20):
        n = int(rng.integers(1, 50))
        pk = oracle.mixed_packets(n)
        pk["len"] = rng.integers(0, 70000, n)
        pk["len"][rng.random(n) < 0.2] = 0
        pk["out_idx"] = pk["out_idx"][::-1].copy()
        live = pk[pk["len"] > 0]
        want = oracle.total_checksums(live) if live.size else 0
        assert hdfs.total_checksums(pk) == want


def _cases():
    yield "c2_shape", oracle.uniform_packets(64)
    yield "mixed", oracle.mixed_packets(24)
    yield "ragged", oracle.uniform_packets(9, pkt_len=65436, stride=65536)
    odd = np.zeros(6, oracle.PACKET_DTYPE)
    odd["payload_off"] = [0, 5, 20000, 30001, 40000, 50000]
    odd["len"] = [4999, 3000, 7000, 3, 1, 9000]
    odd["bpc"] = [512, 512, 100, 512, 1024, 1536]
    odd["out_idx"] = np.cumsum([0] + [(l + b - 1) // b for l, b in zip(odd["len"][:-1], odd["bpc"][:-1])])
    yield "odd", odd
    # padded power-of-two tiles (bpc = 512 * 2^lg - pad), with and without
    # tails, a first chunk too close to the buffer start for the early loads
    pad_pk = np.zeros(9, oracle.PACKET_DTYPE)
    pad_pk["payload_off"] = [3, 9000, 30000, 70000, 80017, 120000, 140000, 200000, 300000]
    pad_pk["len"] = [5000, 20000, 33000, 9000, 40000, 16380, 65536, 65536, 70000]
    pad_pk["bpc"] = [1000, 700, 2000, 100, 4000, 8000, 1000, 511, 8191]
    pad_pk["out_idx"] = np.cumsum([0] + [(l + b - 1) // b for l, b in zip(pad_pk["len"][:-1], pad_pk["bpc"][:-1])])
    yield "padded", pad_pk


@pytest.mark.parametrize("name,pk", list(_cases()))
def test_plan_covers_every_chunk_once(hdfs, orc, name, pk):
    """Re-derive every checksum from the work items alone (CPU) and compare."""
    tiles, gen = hdfs.debug_plan(pk)
    extent = int((pk["payload_off"] + pk["len"]).max())
    payload = oracle.xorshift64_bytes(extent + 64, 77)
    n = oracle.total_checksums(pk)
    want = orc.batch(payload, pk, n)
    got = np.full(n, 0xDEADBEEF, np.uint32)
    seen = np.zeros(n, np.int32)
    for t in tiles:
        meta, src, tl = int(t["meta"]), int(t["src"]) & ((1 << 48) - 1), int(t["src"]) >> 48
        if meta & 0xC0000000 == 0x40000000:  # half tile: n chunks of M blocks + a partial half block each
            nch, m, padh = meta & 0xFF, (meta >> 8) & 0xFF, (meta >> 18) & 511
            bpc = 512 * m + 256 - padh
            assert m in (0, 1, 2) and 1 <= nch <= (32, 10, 6)[m] and padh < 256 and tl == 0 and bpc >= 4
            assert padh == 0 or src >= 16
        elif meta & 0x80000000:  # general tile: nch chunks of any bpc in [4, 8192], k virtual blocks each
            k, nch, pad = (meta >> 8) & 31, (meta >> 13) & 31, (meta >> 18) & 511
            bpc, kt = k * 512 - pad, (tl + 511) // 512
            assert meta & 0xFF == (nch * k + kt + 15) // 16 and 1 <= nch <= 16 and 4 <= bpc <= 8192 and pad < 512
            assert bpc & (bpc - 1) or bpc < 512 or tl  # powers of two >= 512: power-of-two tiles, but the
            #                                           last one of a packet with a tail chunk is general
            assert pad == 0 or src >= 16  # padded loads start up to 15 bytes early
            assert tl == 0 or 4 <= tl < bpc  # a packet's tail chunk after the full ones
        else:
            nb, lg, pad = meta & 0xFF, (meta >> 8) & 0xFF, (meta >> 18) & 511
            assert 1 <= nb <= 16 and nb % (1 << lg) == 0 and tl == 0  # any alignment (unaligned tile loads)
            assert meta & ~(0xFFFF | (511 << 18)) == 0 and lg <= 4
            # padded power-of-two tiles: chunks of 512 << lg minus pad bytes
            assert pad == 0 or (src >= 16 and (512 << lg) - pad >= 4)  # (pad < 512: k = ceil(bpc / 512))
            bpc, nch = (512 << lg) - pad, nb >> lg
        for c in range(nch + (1 if tl else 0)):
            s = src + c * bpc
            got[int(t["out"]) + c] = orc.crc32c(payload[s:s + (bpc if c < nch else tl)])
            seen[int(t["out"]) + c] += 1
    for g in gen:
        s = int(g["src"])
        got[int(g["out"])] = orc.crc32c(payload[s:s + int(g["len"])])
        seen[int(g["out"])] += 1
    assert np.all(seen == 1)
    assert np.array_equal(got, want)


def test_plan_fast_path_shapes(hdfs):
    tiles, gen = hdfs.debug_plan(oracle.uniform_packets(4096))
    assert tiles.size == 4096 * 8 and gen.size == 0 and np.all(tiles["meta"] == 16)
    tiles, gen = hdfs.debug_plan(oracle.mixed_packets(3))
    assert list(tiles["meta"][:1]) == [16] and set(int(m) >> 8 for m in tiles["meta"]) == {0, 1, 3}
    # a tail of at most 512 bytes is a GenItem of its own (the tiles stay power-of-two ones) ...
    tiles, gen = hdfs.debug_plan(oracle.uniform_packets(1, pkt_len=65436))
    assert gen.size == 1 and int(gen["len"][0]) == 65436 % 512 and not np.any(tiles["meta"] >> 31)
    # ... a longer one rides in the last tile, which becomes a general item
    pk = oracle.uniform_packets(1, pkt_len=65436)
    pk["bpc"] = 1024
    tiles, gen = hdfs.debug_plan(pk)
    assert gen.size == 0 and int(tiles["src"][-1]) >> 48 == 65436 % 1024 and int(tiles["meta"][-1]) >> 31
    tiles, gen = hdfs.debug_plan(oracle.uniform_packets(1, pkt_len=65539))  # a 3-byte tail: general path
    assert gen.size == 1 and int(gen["len"][0]) == 3
    # bpc 1000 (k = 2, pad 24): 65 full chunks and a 536-byte tail -> 8 padded
    # tiles of 8 chunks, then one general item of the last chunk + the tail
    pk = oracle.uniform_packets(1)
    pk["bpc"], pk["payload_off"] = 1000, 64  # (a first chunk at offset < 16 would be a GenItem)
    tiles, gen = hdfs.debug_plan(pk)
    meta = tiles["meta"].astype(np.int64)
    assert gen.size == 0 and tiles.size == 9
    assert list(meta[:8]) == [16 | (1 << 8) | (24 << 18)] * 8 and meta[8] >> 31 and (meta[8] >> 13) & 31 == 1
    # half tiles: bpc 700 (M = 1) -> 93 chunks and a 436-byte tail: 9 tiles of
    # 10 chunks, one general item of 3 chunks + the tail; bpc 100 (M = 0): 655
    # chunks and a 36-byte tail: 20 tiles of 32, one general item of 15 + tail
    for bpc, ntiles, mhead, rest in ((700, 9, 10 | (1 << 8) | (68 << 18), 3), (100, 20, 32 | (156 << 18), 15)):
        pk = oracle.uniform_packets(1)
        pk["bpc"], pk["payload_off"] = bpc, 64
        tiles, gen = hdfs.debug_plan(pk)
        meta = tiles["meta"].astype(np.int64)
        assert gen.size == 0 and tiles.size == ntiles + 1, bpc
        assert list(meta[:ntiles]) == [0x40000000 | mhead] * ntiles, bpc
        assert meta[ntiles] >> 31 and (meta[ntiles] >> 13) & 31 == rest, bpc
    # no tail: every chunk in padded tiles (bpc 4000, k = 8: 2 chunks per tile)
    pk = oracle.uniform_packets(1, pkt_len=64000)
    pk["bpc"], pk["payload_off"] = 4000, 64
    tiles, gen = hdfs.debug_plan(pk)
    assert gen.size == 0 and tiles.size == 8 and np.all(tiles["meta"] == 16 | (3 << 8) | (96 << 18))


@pytest.fixture(scope="module")
def model(hdfs):
    img, c_lg, c_small = hdfs.debug_lds_image()
    return KernelModel(img, c_lg, c_small)


def test_affine_constants(hdfs, orc, model):
    for lg in range(5):
        assert model.c_lg[lg] == orc.crc32c(np.zeros(512 << lg, np.uint8))
    for r in range(4):
        assert model.c_small[r] == orc.crc32c(np.zeros(r, np.uint8))


@pytest.mark.parametrize("lg", [0, 1, 2, 3, 4])
def test_kernel_model_fast_tiles(orc, model, lg):
    bpc = 512 << lg
    data = oracle.xorshift64_bytes(bpc * 6, 100 + lg)
    data[:bpc] = 0
    data[bpc:2 * bpc] = 0xFF
    got = model.fast_chunks(data, lg)
    want = orc.chunks(data, bpc)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("bpc", [4, 100, 511, 513, 700, 1000, 1023, 1537, 2000, 3585, 4000, 7681, 8191])
def test_kernel_model_padded_tiles(orc, model, bpc):
    """Padded power-of-two tiles: each chunk right-aligned into its 2^lg
    virtual blocks behind pad zeros, reduced like a power-of-two chunk, with
    crc(0, zeros(bpc)) as the affine constant instead of 512 << lg's."""
    lg = max(0, (bpc - 1).bit_length() - 9)
    k = 1 << lg
    pad = 512 * k - bpc
    assert 0 < pad < 512
    data = oracle.xorshift64_bytes(bpc * 5, 300 + bpc)
    data[bpc:2 * bpc] = 0xFF
    virt = np.zeros((5, 512 * k), np.uint8)
    virt[:, pad:] = data.reshape(5, bpc)
    got = model.fast_chunks(virt.reshape(-1), lg) ^ np.uint32(model.c_lg[lg]) ^ np.uint32(
        orc.crc32c(np.zeros(bpc, np.uint8)))
    assert np.array_equal(got, orc.chunks(data, bpc))


@pytest.mark.parametrize("bpc", [4, 17, 100, 255, 256, 513, 600, 700, 767, 768, 1025, 1100, 1280])
def test_kernel_model_half_tiles(orc, model, bpc):
    """Half tiles: a chunk's partial part (bpc - 512 M <= 256 bytes) right-
    aligned into the upper half of a zero block -- what a lane of the lower
    half computes with the columns q + 16 -- then, for M >= 1, shifted by
    Z^(512 M) past the chunk's full blocks."""
    m = bpc // 512
    r = bpc - 512 * m
    data = oracle.xorshift64_bytes(bpc * 3, 700 + bpc)
    for c in range(3):
        chunk = data[c * bpc:(c + 1) * bpc]
        half = np.zeros(512, np.uint8)
        half[512 - r:] = chunk[:r]
        x = int(model.block_lin(half.reshape(1, 512))[0])
        if m:  # the partial half shifted past the chunk's M full blocks, which are joined like a chunk's
            x = model.zshift(m, x)
            for j in range(m):
                b = int(model.block_lin(chunk[r + 512 * j:r + 512 * (j + 1)].reshape(1, 512))[0])
                x ^= model.zshift(m - 1 - j, b) if m - 1 - j else b
        assert x ^ orc.crc32c(np.zeros(bpc, np.uint8)) == orc.crc32c(chunk), (bpc, c)


def test_kernel_model_general_chunks(orc, model):
    buf = oracle.xorshift64_bytes(20000, 55)
    for n in [1, 2, 3, 4, 5, 15, 16, 17, 100, 411, 511, 512, 513, 1000, 1536, 4095, 8192, 9001]:
        assert model.general_chunk(buf[:n]) == orc.crc32c(buf[:n]), n
    for n in [1, 3, 4, 700]:
        assert model.general_chunk(np.zeros(n, np.uint8)) == orc.crc32c(np.zeros(n, np.uint8))


@pytest.mark.parametrize("bpc", [4, 5, 100, 511, 513, 1000, 1536, 2560, 4000, 7680, 8191])
def test_kernel_model_general_tiles(hdfs, orc, bpc):
    """General tiles: each chunk right-aligned into k = ceil(bpc / 512)
    virtual blocks (zero prefix, no pre-inversion in the data), block b
    shifted by Z^(512 (k - 1 - b)) from the S4 image's shift section, XORed,
    ^ crc(0, zeros(bpc)) -- the affine constant the kernel reads from the
    zero-crc table (crc_math.h zero_crc_table)."""
    m4 = KernelModelS4(hdfs.debug_lds_image_s4())
    img, c_lg, c_small = hdfs.debug_lds_image()
    zm = KernelModel(img, c_lg, c_small)
    k = (bpc + 511) // 512
    pad = k * 512 - bpc
    data = oracle.xorshift64_bytes(bpc * 5, bpc)
    data[:bpc] = 0
    zero_crc = orc.crc32c(np.zeros(bpc, np.uint8))
    got = []
    for c in range(5):
        v = np.zeros(k * 512, np.uint8)
        v[pad:] = data[c * bpc:(c + 1) * bpc]
        lins = m4.block_lin(v.reshape(k, 512))
        x = 0
        for j in range(k):
            s = k - 1 - j
            x ^= zm.zshift(s, int(lins[j])) if s else int(lins[j])
        got.append(x ^ zero_crc)
    assert np.array_equal(np.array(got, np.uint32), orc.chunks(data, bpc))


def test_write_plan_decomposition(hdfs):
    """crc32c_plan_create_buffers' work items (hadooprpc.c:666-725 packet
    assembly): an all-NULL 4 MiB ftruncate extension is constant runs only (no
    payload read); the four FUSE write buffers give tiles inside each data
    buffer, seg items only for chunks spanning a buffer boundary, and
    constants for chunks of zero fill."""
    MB4 = 4 << 20
    c = hdfs.debug_write_plan([(0, MB4)], 0, MB4)
    assert c == {"tiles": 0, "gen": 0, "seg": 0, "pieces": 0, "consts": 8, "nchecksums": 8192}
    base = 1 << 40  # device addresses are opaque to the plan builder
    # TRUNCATE 1000 B of old data, NULLPADDING 3000, THEDATA 70000, TRAILINGDATA 5000
    bufs = [(base, 1000), (0, 3000), (base + (1 << 20), 70000), (base + (2 << 20), 5000)]
    c = hdfs.debug_write_plan(bufs, 0, 79000, blockoffset=0)
    n = sum((ln + 511) // 512 for ln in hdfs.packetize(79000, 0, 65536, 512))
    assert c["nchecksums"] == n == (65536 // 512) + (79000 - 65536 + 511) // 512
    # chunk 1 (1000 / 3000 boundary) and the chunks at 4000 and 74000 span buffers
    assert c["seg"] == 3 and c["pieces"] == 4
    assert c["consts"] == 1  # chunks 2..6: zero fill only (bytes 1024 .. 3583)
    # an unaligned block offset: the first packet finishes one chunk (hadooprpc.c:832-840)
    c = hdfs.debug_write_plan(bufs, 100, 5000, blockoffset=700)
    assert c["nchecksums"] == sum((ln + 511) // 512 for ln in hdfs.packetize(5000, 700, 65536, 512))
    with pytest.raises(hdfs.Crc32cError):
        hdfs.debug_write_plan(bufs, 0, 79001)  # beyond the buffers


def test_gpu_entry_points_fail_loudly_without_gpu(hdfs):
    if hdfs.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(hdfs.Crc32cError) as ei:
        hdfs.Context(0)
    assert ei.value.rc == -19  # -ENODEV: no CPU substitute behind the GPU API
    with pytest.raises(hdfs.Crc32cError):
        hdfs.chunks(np.zeros(1024, np.uint8), 512)
    assert hdfs.last_path() == hdfs.PATH_NONE


def test_cpu_fallback_is_opt_in_and_observable(hdfs, orc):
    """SURVEY.md section 5's failure contract, as an explicit flag: without a
    GPU, crc32c_chunks / crc32c_batch_host given CRC32C_CPU_FALLBACK finish
    on the product's host path (crc32c_chunks_cpu) and crc32c_last_path()
    says so; without the flag they fail (-ENODEV)."""
    if hdfs.device_count() > 0:
        pytest.skip("a GPU is visible")
    pkt = oracle.xorshift64_bytes(70000, 12)
    F = hdfs.CRC32C_CPU_FALLBACK
    assert np.array_equal(hdfs.chunks(pkt, 512, F), orc.chunks(pkt, 512))
    assert hdfs.last_path() == hdfs.PATH_CPU
    assert np.array_equal(hdfs.chunks(pkt, 1000, F | hdfs.CRC32C_BIG_ENDIAN), orc.chunks(pkt, 1000, True))
    with pytest.raises(hdfs.Crc32cError):
        hdfs.chunks(pkt, 512)
    assert hdfs.last_path() == hdfs.PATH_NONE


def test_s4_image_matches_nibble_image(hdfs, model):
    """The slicing-by-4 image (byte tables replicated per lane column, the
    per-column finishing operators N_q, the Z^(512 s) section) computes the
    same block lin() as the positional nibble image."""
    img4 = hdfs.debug_lds_image_s4()
    m4 = KernelModelS4(img4)
    for t in m4.t:  # every column holds the same byte table
        assert (t == t[:, :1]).all()
    rng = np.random.default_rng(11)
    blocks = rng.integers(0, 256, (64, 512), dtype=np.uint8)
    blocks[0] = 0
    blocks[1] = 0xFF
    assert np.array_equal(m4.block_lin(blocks), model.block_lin(blocks))
    img, _, _ = hdfs.debug_lds_image()
    w4 = img4.view("<u4")
    w = img.view("<u4")
    assert np.array_equal(w4[KernelModelS4.SHIFT_OFF // 4:], w[65536 // 4:65536 // 4 + w4.size - KernelModelS4.SHIFT_OFF // 4])


# ---- CHECKSUM_CRC32 (zlib polynomial) ------------------------------------
def test_hdfs_crc32_matches_zlib(hdfs):
    import zlib

    assert hdfs.hdfs_crc32(b"123456789") == 0xCBF43926  # the CRC-32 check value
    assert hdfs.hdfs_crc32(b"") == 0
    rng = np.random.default_rng(5)
    buf = rng.integers(0, 256, 70000, dtype=np.uint8)
    for off, n in [(0, 1), (1, 7), (3, 8), (5, 513), (0, 65536), (7, 69993)]:
        assert hdfs.hdfs_crc32(buf[off:off + n]) == zlib.crc32(buf[off:off + n].tobytes()), (off, n)
    # incremental, as crc32c(crc, ...)
    assert hdfs.hdfs_crc32(buf[100:300], hdfs.hdfs_crc32(buf[:100])) == zlib.crc32(buf[:300].tobytes())


@pytest.mark.parametrize("lg", [0, 2, 4])
def test_crc32_tables_match_zlib(hdfs, lg):
    """The CRC32 images (nibble and S4) and constants give zlib's per-chunk CRC32."""
    img, _, _ = hdfs.debug_lds_image()  # layout only; CRC32 contents below
    c_lg, c_small = hdfs.debug_affine_constants(hdfs.CRC32C_TYPE_CRC32)
    img4 = hdfs.debug_lds_image_s4(hdfs.CRC32C_TYPE_CRC32)
    m4 = KernelModelS4(img4)
    bpc = 512 << lg
    data = oracle.xorshift64_bytes(bpc * 4, 300 + lg)
    data[:bpc] = 0
    lins = m4.block_lin(data.reshape(-1, 512)).reshape(-1, 1 << lg)
    # combine the blocks of a chunk with Z^(512 s) from the image's shift section
    zm = KernelModel(np.concatenate([np.zeros(65536, np.uint8), img4[KernelModelS4.SHIFT_OFF:]]), c_lg, c_small)
    got = []
    for c in range(lins.shape[0]):
        x = 0
        for m in range(1 << lg):
            s = (1 << lg) - 1 - m
            x ^= zm.zshift(s, int(lins[c, m])) if s else int(lins[c, m])
        got.append(x ^ int(c_lg[lg]))
    assert np.array_equal(np.array(got, np.uint32), oracle.zlib_chunks(data, bpc))
    for r in range(4):
        import zlib
        assert int(c_small[r]) == zlib.crc32(bytes(r))
    assert img.size > 0


def test_workloads_match_oracle_shapes(hdfs):
    """The bench's synthetic batches (native-hdfs-fuse_amd/workloads.py) have
    the same packet layout as the oracle's helpers the fixtures were made
    with."""
    from hdfs_crc32c_amd import workloads

    for n in (1, 64, 4096):
        assert np.array_equal(workloads.uniform_packets(n), oracle.uniform_packets(n))
        assert np.array_equal(workloads.mixed_packets(n), oracle.mixed_packets(n))
    assert np.array_equal(workloads.uniform_packets(9, pkt_len=65436, stride=65536),
                          oracle.uniform_packets(9, pkt_len=65436, stride=65536))
    for name in ("c2", "c3", "c5", "p17"):
        pk, text = workloads.config_packets(name)
        assert pk.dtype == hdfs.PACKET_DTYPE and text
    a, b = workloads.synthetic_bytes(1000, 3), workloads.synthetic_bytes(1000, 3)
    assert a.dtype == np.uint8 and np.array_equal(a, b)


def test_no_device_wide_sync_on_plan_paths():
    """Plan blocks are recycled after per-stream events, not a device-wide
    synchronisation: hipDeviceSynchronize appears in the runtime only in the
    context teardown (release_pools, and there only for blocks a graph
    captured), never on a plan create / exec / destroy path (which would wait
    for every stream of the device and break a global-mode graph capture on
    another thread)."""
    csrc = os.path.join(ROOT, "native-hdfs-fuse_amd", "csrc")
    sig = re.compile(r"^(?:[A-Za-z_][\w:<>\*&]*\s+)+\**([A-Za-z_]\w*)\(", re.M)
    for name in ("crc32c_runtime.hip", "crc32c_multi.hip", "crc32c_kernel.hip"):
        text = re.sub(r"//[^\n]*", "", open(os.path.join(csrc, name)).read())
        for m in re.finditer(r"hipDeviceSynchronize", text):
            funcs = [f.group(1) for f in sig.finditer(text[:m.start()])]
            assert funcs and funcs[-1] == "release_pools", (name, funcs[-1:])
    text = open(os.path.join(csrc, "runtime_internal.h")).read()
    assert "kEpochBlocks" not in text


def test_product_library_loads_rccl_only_for_multi_gpu(hdfs):
    """A single-GPU caller (the FUSE write path) needs no RCCL at load time:
    the product library does not link librccl; crc32c_multi.hip loads it by
    SONAME on first use (sharing the copy torch already holds)."""
    import subprocess

    needed = subprocess.run(["readelf", "-d", hdfs.LIB_PATH], capture_output=True, text=True).stdout
    assert "NEEDED" in needed and "rccl" not in needed, needed
    assert b"librccl.so.1" in open(hdfs.LIB_PATH, "rb").read()


def test_kernel_buffer_resources_not_sign_extended(tmp_path):
    """Regression guard (round 3): the payload loads' buffer resources are
    built from SGPRs by uniform_rsrc (crc32c_device.h).  A first version
    widened readfirstlane's int result directly, so a base address whose low
    word was >= 2^31 sign-extended over the high word (an s_bfe_i64 of the
    address into the resource) and the kernel faulted on such buffers.  The
    production kernels' device assembly must contain no 64-bit sign
    extension of that kind."""
    import subprocess

    csrc = os.path.join(ROOT, "native-hdfs-fuse_amd", "csrc")
    out = str(tmp_path / "k.s")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", "-I" + os.path.join(ROOT, "include"), "-I" + csrc,
                        os.path.join(csrc, "crc32c_kernel.hip"), "-o", out], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    asm = open(out).read()
    assert "hdfs_crc32c_plan_kernel" in asm
    assert not re.search(r"s_bfe_i64\s+s\[\d+:\d+\], s\[\d+:\d+\], 0x200000", asm)
    # and no waterfall (readfirstlane + execnz) loop around a payload load
    lines = asm.split("\n")
    for i, line in enumerate(lines):
        if "buffer_load_dwordx4" in line:
            window = lines[max(0, i - 12):i + 4]
            assert not (any("v_readfirstlane" in w for w in window) and any("s_cbranch_execnz" in w for w in window)), i


def test_plan_keeps_stream_objects_alive():
    """Plan.exec/verify accept a stream object and hold it until close() (destroy touches
    the plan's launch streams, crc32c_plan_destroy in include/hdfs_crc32c.h)."""
    import importlib
    pkg = importlib.import_module("native-hdfs-fuse_amd")

    class FakeStream:
        cuda_stream = 0x1234

    p = pkg.Plan.__new__(pkg.Plan)
    p.handle = None
    p._streams = {}
    s = FakeStream()
    assert p._stream(s) == 0x1234 and p._stream(7) == 7
    # (None = the default stream, numpy integers are handles too)
    import numpy as np
    assert p._stream(None) == 0 and p._stream(np.int64(9)) == 9 and p._stream(np.uint64(11)) == 11
    assert p._streams == {0x1234: s}
    p.close()
    assert p._streams == {}
    mp = pkg.MultiPlan.__new__(pkg.MultiPlan)  # (MultiPlan.exec keeps its stream objects the same way)
    mp.handle = None
    mp._streams = {}
    assert pkg._stream_handle(s, mp._streams) == 0x1234 and mp._streams == {0x1234: s}
    mp.close()
    assert mp._streams == {}
