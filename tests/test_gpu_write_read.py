"""GPU parity of round 2's paths: general tiles (any bytesPerChecksum), packet
assembly from Hadoop_Fuse_Buffer lists with NULL = zero fill
(crc32c_plan_create_buffers), received-frame verification
(crc32c_verify_frames_host), and the multi-GPU plan with its RCCL gather
(crc32c_multi_plan_*).  Everything runs through the C ABI; the oracle is the
checker."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import oracle
from conftest import golden_batch_packets

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch


def _expected_write(orc, stream: np.ndarray, bufferoffset, length, blockoffset, packetsize, bpc, big_endian=False):
    """hadoop_rpc_send_packets' checksums over the assembled stream (oracle):
    packets as crc32c_packetize cuts them, chunks from each packet's start."""
    out, pos, sent = [], bufferoffset, 0
    while True:
        plen = min(length - sent, packetsize)
        past = (blockoffset + sent) % bpc
        if plen > 0 and past:
            plen = min(bpc - past, length - sent)
        if plen == 0:
            break
        out.append(orc.chunks(stream[pos:pos + plen], bpc, big_endian))
        pos += plen
        sent += plen
    return np.concatenate(out) if out else np.zeros(0, np.uint32)


def _run_plan(plan, n, stream, payload=0):
    torch = _torch()
    out = torch.full((max(n, 1),), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    plan.exec(payload, out.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    return out.cpu().numpy().view(np.uint32)[:n]


def _verify(plan, expected: np.ndarray, stream, payload=0):
    torch = _torch()
    exp = torch.from_numpy(expected.view(np.int32).copy()).cuda()
    res = torch.zeros(2, dtype=torch.int32, device="cuda")
    plan.verify(payload, exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    return res.cpu().numpy().view(np.uint32).tolist()


# ---- general tiles -----------------------------------------------------------
@pytest.mark.parametrize("bpc", [4, 7, 100, 511, 513, 1000, 1536, 2560, 3072, 4000, 6144, 7680, 8191])
def test_general_tiles_any_bpc(hdfs, gpu_ctx, orc, bpc):
    """Packets of bpc outside 512 * 2^k take general tiles (16 // k chunks of k
    virtual blocks), or padded power-of-two tiles where k is a power of two
    (the packet's tail still in a general tile): at offset 0 (padded tiles fall back to the general path
    only for the first chunk), at every phase mod 16, with ragged tails; exec
    and verify against the oracle."""
    torch = _torch()
    rows, off, out = [], 0, 0
    tails = [4, 5, 100, 508, 509, 511, 513, 1000, 1023, 1025, 4097]  # the tail chunk rides in the last tile
    for i in range(20):
        ln = 65536 - (0 if i % 3 else 777)
        if i % 3 == 2:
            ln = 65536 // bpc * bpc - bpc + tails[i % len(tails)] % bpc
        rows.append((off, out, ln, bpc))
        out += (ln + bpc - 1) // bpc
        off += ln + (i % 16) + 1
    pk = np.array(rows, hdfs.PACKET_DTYPE)
    tiles, gen = hdfs.debug_plan(pk)
    meta = tiles["meta"].astype(np.int64)
    assert np.any(meta >> 31) or np.any((meta >> 18) & 511)  # general or padded power-of-two tiles
    if 16 <= bpc <= 7680:  # (8191: a 16-block chunk leaves a tile no room)
        assert np.any(tiles["src"] >> np.uint64(48))  # tails in tiles
    payload = oracle.xorshift64_bytes(off + 64, 3000 + bpc)
    payload[:bpc * 2] = 0  # a zero chunk
    want = orc.batch(payload, pk, out)
    dev = torch.from_numpy(payload).cuda()
    stream = torch.cuda.current_stream()
    plan = hdfs.Plan(gpu_ctx, pk)
    assert np.array_equal(_run_plan(plan, out, stream, dev.data_ptr()), want)
    assert _verify(plan, want, stream, dev.data_ptr()) == [0, 0xFFFFFFFF]
    bad = want.copy()
    bad[[out // 3, out - 2]] ^= 0x800
    assert _verify(plan, bad, stream, dev.data_ptr()) == [2, out // 3]
    plan.close()


@pytest.mark.parametrize("bpc", [100, 1000, 1536, 2560, 3000, 5000, 7000])
def test_general_items_subtile_spans(hdfs, gpu_ctx, orc, bpc):
    """Every chunk count 1..17 of a general item with tails of every block
    count, so that full chunks and the tail chunk start, end and span 16-block
    subtile boundaries at every position (padded and unpadded); one batch,
    exec and verify against the oracle."""
    torch = _torch()
    rows, off, out = [], 64, 0
    for nfull in range(1, 18):
        for tl in (0, 4, 100, 509, 511, 513, 1000, 1283, 1532, 2047, 4100, 6000):
            if tl >= bpc:
                continue
            ln = nfull * bpc + tl
            rows.append((off, out, ln, bpc))
            out += (ln + bpc - 1) // bpc
            off += ln + (1 if nfull % 5 == 0 else 16 - ln % 16)
    pk = np.array(rows, hdfs.PACKET_DTYPE)
    tiles, gen = hdfs.debug_plan(pk)
    assert np.any(tiles["src"] >> np.uint64(48)) and np.any((tiles["meta"] & 0xFF) > 1)
    payload = oracle.xorshift64_bytes(off + 64, 4000 + bpc)
    want = orc.batch(payload, pk, out)
    dev = torch.from_numpy(payload).cuda()
    stream = torch.cuda.current_stream()
    plan = hdfs.Plan(gpu_ctx, pk)
    got = _run_plan(plan, out, stream, dev.data_ptr())
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    assert _verify(plan, want, stream, dev.data_ptr()) == [0, 0xFFFFFFFF]
    plan.close()


def test_general_tiles_device_addresses_near_page_start(hdfs, gpu_ctx, orc):
    """CRC32C_DEVICE_ADDRESSES plans with padded general tiles: packets
    starting 0..20 bytes into a fresh allocation (padded tiles load up to 15
    bytes before a chunk, allowed only inside the same 4 KiB page)."""
    torch = _torch()
    bufs, rows, want, out = [], [], [], 0
    for k in range(21):
        data = oracle.xorshift64_bytes(40000 + 64, 50 + k)
        t = torch.from_numpy(data).cuda()
        bufs.append(t)
        bpc = (100, 1000, 1536, 700)[k % 4]
        ln = 40000 - k
        rows.append((t.data_ptr() + k, out, ln, bpc))
        want.append(orc.chunks(data[k:k + ln], bpc))
        out += (ln + bpc - 1) // bpc
    pk = np.array(rows, hdfs.PACKET_DTYPE)
    plan = hdfs.Plan(gpu_ctx, pk, hdfs.CRC32C_DEVICE_ADDRESSES)
    stream = torch.cuda.current_stream()
    assert np.array_equal(_run_plan(plan, out, stream), np.concatenate(want))
    plan.close()


# ---- packet assembly from buffer lists (hadooprpc.c:666-725) -----------------
def _fuse_write_buffers(torch, rng, lens, null_mask, seed):
    """Device buffers of the given lengths (None where NULL), and the host
    stream they assemble to."""
    bufs, devs, parts = [], [], []
    for i, (n, is_null) in enumerate(zip(lens, null_mask)):
        if is_null:
            bufs.append((0, n))
            parts.append(np.zeros(n, np.uint8))
        else:
            d = oracle.xorshift64_bytes(n + 32, seed + i)
            skew = int(rng.integers(0, 16))
            t = torch.from_numpy(d).cuda()
            devs.append(t)
            bufs.append((t.data_ptr() + skew, n))
            parts.append(d[skew:skew + n])
    return bufs, devs, np.concatenate(parts) if parts else np.zeros(0, np.uint8)


@pytest.mark.parametrize("shape", ["truncate_pad_data_trailing", "data_only", "pad_then_data", "tiny_pieces",
                                   "unaligned_block_offset", "bpc_1536", "crc32_big_endian"])
def test_write_plan_four_buffers(hdfs, gpu_ctx, orc, shape):
    """The buffer shapes of hadoop_fuse_write (fuse.c:1348-1354): TRUNCATE
    (old data), NULLPADDING (zeros), THEDATA (the write), TRAILINGDATA (old
    data after it), cut into packets by hadoop_rpc_send_packets
    (hadooprpc.c:815-860) from a block offset; bit-exact against the oracle
    over the assembled stream, exec and verify."""
    torch = _torch()
    rng = np.random.default_rng(sum(shape.encode()))
    bpc, flags, blockoffset, bufferoffset = 512, 0, 0, 0
    if shape == "truncate_pad_data_trailing":
        lens, nulls = [10000, 300000, 1 << 20, 77777], [False, True, False, False]
    elif shape == "data_only":
        lens, nulls = [4 << 20], [False]
    elif shape == "pad_then_data":
        lens, nulls = [12345, 100000], [True, False]
    elif shape == "tiny_pieces":
        lens, nulls = [3, 1, 700, 5, 2000, 1, 9], [False, True, False, True, False, False, True]
    elif shape == "unaligned_block_offset":
        lens, nulls = [5000, 20000, 200000, 3000], [False, True, False, False]
        blockoffset, bufferoffset = 1000 + 37, 333
    elif shape == "bpc_1536":
        lens, nulls = [10000, 4096, 300000, 6000], [False, True, False, False]
        bpc, blockoffset = 1536, 1536 * 3
    else:
        lens, nulls = [10000, 300000, 1 << 20, 77777], [False, True, False, False]
        flags = hdfs.CRC32C_TYPE_CRC32 | hdfs.CRC32C_BIG_ENDIAN
    bufs, devs, stream_bytes = _fuse_write_buffers(torch, rng, lens, nulls, 900)
    length = stream_bytes.size - bufferoffset - 11
    plan = gpu_ctx.write_plan(bufs, bufferoffset, length, blockoffset, 65536, bpc, flags)
    if flags & hdfs.CRC32C_TYPE_CRC32:
        want, pos, sent = [], bufferoffset, 0
        for plen in hdfs.packetize(length, blockoffset, 65536, bpc):
            if plen:
                want.append(oracle.zlib_chunks(stream_bytes[pos:pos + plen], bpc).byteswap())
            pos += plen
        want = np.concatenate(want)
    else:
        want = _expected_write(orc, stream_bytes, bufferoffset, length, blockoffset, 65536, bpc)
    assert plan.nchecksums == want.size
    s = torch.cuda.current_stream()
    got = _run_plan(plan, want.size, s)
    assert np.array_equal(got, want)
    assert _verify(plan, want, s) == [0, 0xFFFFFFFF]
    bad = want.copy()
    bad[want.size // 2] ^= 1
    assert _verify(plan, bad, s) == [1, want.size // 2]
    plan.close()


def test_write_plan_ftruncate_extend_reads_nothing(hdfs, gpu_ctx, orc):
    """ftruncate growing a file by a whole 4 MiB block is a write of NULL
    buffers (fuse.c:1137-1142): every checksum is a plan-time constant
    (crc32c of 512 zero bytes = 30fcedc0), written without reading payload;
    a ragged extension ends with the short zero chunk's constant."""
    torch = _torch()
    s = torch.cuda.current_stream()
    n4 = 4 << 20
    counts = hdfs.debug_write_plan([(0, n4)], 0, n4)
    assert counts["tiles"] == counts["gen"] == counts["seg"] == 0
    plan = gpu_ctx.write_plan([(0, n4)], 0, n4)
    got = _run_plan(plan, 8192, s)
    assert np.all(got == 0x30FCEDC0)
    assert _verify(plan, got, s) == [0, 0xFFFFFFFF]
    plan.close()
    plan = gpu_ctx.write_plan([(0, 1000001)], 0, 1000001, blockoffset=4096)
    want = _expected_write(orc, np.zeros(1000001, np.uint8), 0, 1000001, 4096, 65536, 512)
    assert np.array_equal(_run_plan(plan, want.size, s), want)
    plan.close()


def test_write_plan_random_buffer_lists(hdfs, gpu_ctx, orc):
    """Random buffer lists (1-6 buffers, NULL or data, lengths 0..200000,
    any skew), random bufferoffset / len / blockoffset / bpc / packetsize."""
    torch = _torch()
    rng = np.random.default_rng(77)
    s = torch.cuda.current_stream()
    for trial in range(12):
        nb = int(rng.integers(1, 7))
        lens = [int(x) for x in rng.integers(0, 200000, nb)]
        nulls = [bool(x) for x in rng.random(nb) < 0.3]
        bufs, devs, sb = _fuse_write_buffers(torch, rng, lens, nulls, 2000 + 10 * trial)
        total = sb.size
        bo = int(rng.integers(0, total // 3 + 1))
        length = int(rng.integers(0, total - bo + 1))
        bpc = int(rng.choice([512, 1024, 4096, 100, 1536]))
        blockoffset = int(rng.integers(0, 3)) * int(rng.integers(0, 1 << 20))
        psize = int(rng.choice([65536, bpc * 7]))
        want = _expected_write(orc, sb, bo, length, blockoffset, psize, bpc)
        plan = gpu_ctx.write_plan(bufs, bo, length, blockoffset, psize, bpc)
        assert plan.nchecksums == want.size, trial
        if want.size:
            assert np.array_equal(_run_plan(plan, want.size, s), want), trial
        plan.close()


# ---- received frames (hadooprpc.c:497-584) --------------------------------
def _frames(hdfs, orc, payload, pk, bpc, chunk_offset):
    """A DataNode's packet stream for pk (contiguous from chunk_offset):
    prefixes from crc32c_frame_packets, data behind each."""
    sums = orc.batch(payload, pk, oracle.total_checksums(pk))
    pre, offs = hdfs.frame_packets(pk, sums, 0, block_offset=chunk_offset)
    parts = []
    for i in range(pk.size):
        parts.append(np.frombuffer(pre[int(offs[i]):int(offs[i + 1])], np.uint8))
        o = int(pk["payload_off"][i])
        parts.append(payload[o:o + int(pk["len"][i])])
    return np.concatenate(parts)


@pytest.mark.parametrize("bpc", [512, 4096, 1536])
def test_verify_received_frames(hdfs, gpu_ctx, orc, bpc):
    """A read of 3 MiB + a ragged tail from chunkOffset 8 * bpc: the frame
    run (PLEN|HLEN|header|checksums|data per packet, final empty packet) is
    verified on the GPU without de-interleaving; a flipped data byte and a
    flipped checksum byte are found at the right chunk and offsetInBlock; a
    truncated buffer verifies its whole frames only; a misplaced frame is
    refused."""
    n = 48
    pk = oracle.uniform_packets(n, pkt_len=65536 - 65536 % bpc, bpc=bpc)
    pk["len"][-1] = 12345
    pk = np.concatenate([pk, np.zeros(1, pk.dtype)])  # the block's final empty packet (hadooprpc.c:853-856)
    pk["payload_off"][-1] = pk["payload_off"][-2] + pk["len"][-2]
    pk["bpc"][-1] = bpc
    pk["out_idx"][-1] = oracle.total_checksums(pk[:-1])
    payload = oracle.xorshift64_bytes(int(pk["payload_off"][-1]) + 16, 4242 + bpc)
    chunk_offset = 8 * bpc
    fr = _frames(hdfs, orc, payload, pk, bpc, chunk_offset)
    info, used = hdfs.parse_frames(fr)
    assert info.size == n + 1 and used == fr.size and int(info["last"][-1]) == 1
    r = gpu_ctx.verify_frames(fr, bpc, chunk_offset)
    assert (r.packets, r.data_bytes, r.mismatches, r.first_bad, r.last_packet) == (
        n + 1, int(pk["len"].sum()), 0, 2**64 - 1, 1)
    assert r.checksums == oracle.total_checksums(pk)
    # a flipped data byte in packet 20, chunk 5
    bad = fr.copy()
    at = int(info["data_off"][20]) + 5 * bpc + 17
    bad[at] ^= 0x10
    r = gpu_ctx.verify_frames(bad, bpc, chunk_offset)
    k = int(oracle.total_checksums(pk[:20])) + 5
    assert (r.mismatches, r.first_bad, r.first_bad_offset) == (1, k, chunk_offset + int(pk["payload_off"][20]) + 5 * bpc)
    # a flipped checksum byte of packet 3's first chunk
    bad = fr.copy()
    bad[int(info["sums_off"][3]) + 2] ^= 1
    r = gpu_ctx.verify_frames(bad, bpc, chunk_offset)
    assert (r.mismatches, r.first_bad) == (1, int(oracle.total_checksums(pk[:3])))
    # the first 10.5 frames arrived
    cut = int(info["frame_off"][10]) + 1000
    r = gpu_ctx.verify_frames(fr[:cut], bpc, chunk_offset)
    assert (r.packets, r.consumed, r.mismatches, r.last_packet) == (10, int(info["frame_off"][10]), 0, 0)
    # the DataNode must start at chunkOffset
    with pytest.raises(hdfs.Crc32cError):
        gpu_ctx.verify_frames(fr, bpc, chunk_offset + bpc)


# ---- several GPUs: device-resident plan + RCCL gather (config 4) ------------
@pytest.mark.parametrize("self_send", [False, True])
def test_multi_plan_config4_rccl_gather(hdfs, golden, orc, self_send):
    """Config 4 through crc32c_multi_plan_*: a 128 MiB file as 32 x 4 MiB
    blocks dealt round-robin over the communicator's ranks (here every
    visible device, one process; the box has one), each rank checksumming
    its shard device-resident, every group's checksum range received by RCCL
    straight into its file-order place on rank 0: the golden c4 digest from
    the reference.  With CRC32C_MULTI_SELF_SEND rank 0's own checksums travel
    through RCCL too (a send to itself), so the transport runs on one GPU.
    Then the whole step (kernels + RCCL group) captured into a HIP graph and
    replayed twice, as the bench's config-4 steps are."""
    torch = _torch()
    spec = [b for b in golden["batches"] if b["name"] == "c4_file_128MiB"][0]
    pk = golden_batch_packets(spec)
    payload = oracle.xorshift64_bytes(spec["payload_bytes"], spec["seed"])
    ndev = torch.cuda.device_count()
    m = hdfs.Multi(list(range(ndev)))
    mp = m.plan(pk, 64, hdfs.CRC32C_MULTI_SELF_SEND if self_send else 0)
    assert mp.nchecksums == spec["nchecksums"]
    layout, shard_bytes = hdfs.multi_layout(pk, 64, ndev)
    assert layout.shape == (32, 4) and list(layout[:, 0]) == [g % ndev for g in range(32)]
    shards = []
    for r in range(ndev):
        host = np.zeros(int(shard_bytes[r]) + 16, np.uint8)
        for g in range(32):
            rank, soff, poff, nbytes = (int(x) for x in layout[g])
            if rank == r:
                host[soff:soff + nbytes] = payload[poff:poff + nbytes]
        shards.append(torch.from_numpy(host).to("cuda:%d" % r))
    out = torch.zeros(mp.nchecksums, dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    mp.exec([t.data_ptr() for t in shards], out.data_ptr())
    m.sync()
    got = out.cpu().numpy().view(np.uint32)
    assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == spec["sha256_le"]
    # again, on the caller's streams, after clearing the output
    out.zero_()
    streams = [torch.cuda.Stream(device="cuda:%d" % r) for r in range(ndev)]
    torch.cuda.synchronize()
    mp.exec([t.data_ptr() for t in shards], out.data_ptr(), [s.cuda_stream for s in streams])
    for s in streams:
        s.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), got)
    if ndev == 1:
        cs = torch.cuda.Stream()
        mp.exec([t.data_ptr() for t in shards], out.data_ptr(), [cs.cuda_stream])  # (stream switch outside the capture)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=cs, capture_error_mode="thread_local"):
            for _ in range(3):
                mp.exec([t.data_ptr() for t in shards], out.data_ptr(), [cs.cuda_stream])
        for _ in range(2):
            out.zero_()
            torch.cuda.synchronize()
            graph.replay()
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy().view(np.uint32), got)
        del graph
    mp.close()
    m.close()


@pytest.mark.parametrize("per_group", [False, True], ids=["packed", "per_group"])
def test_multi_plan_self_send_several_transfers_per_peer(hdfs, orc, per_group):
    """ONE sender with several group ranges to place, eagerly and
    graph-captured.  A file of 12 groups whose checksum ranges leave gaps
    between groups (out_idx of group g starts at g (n + 37)): the sender's
    local array is dense, the file-order places are not, so no two
    placements merge.  Packed (the default): one ncclSend / ncclRecv pair to
    self (CRC32C_MULTI_SELF_SEND) into the plan's staging array, then the
    scatter kernel; per group (CRC32C_MULTI_PER_GROUP_RECV): 12 pairs, matched
    in posting order, straight into place.  Every group's checksums land in
    place, the gaps keep their sentinel, also after the stream switches and
    in two graph replays; a second stream object freed before the switch is
    kept alive by the plan (the next exec records an event on it)."""
    import gc

    torch = _torch()
    gp, ngroups, gap = 3, 12, 37
    pk = oracle.uniform_packets(gp * ngroups)
    per = 128 * gp
    pk["out_idx"] = np.array([(i // gp) * (per + gap) + (i % gp) * 128 for i in range(pk.size)], np.uint64)
    ln, xs = hdfs.multi_transfers(pk, gp, 1, hdfs.CRC32C_MULTI_SELF_SEND)
    assert xs.shape == (ngroups, 4) and list(ln) == [per * ngroups]
    payload = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 16, 515)
    total = int((pk["out_idx"] + 128).max())
    want = np.full(total, 0x5A5A5A5A, np.uint32)
    want_idx = np.concatenate([np.arange(g * (per + gap), g * (per + gap) + per) for g in range(ngroups)])
    want[want_idx] = orc.batch(payload, pk, total)[want_idx]
    m = hdfs.Multi([0])
    mp = m.plan(pk, gp, hdfs.CRC32C_MULTI_SELF_SEND | (hdfs.CRC32C_MULTI_PER_GROUP_RECV if per_group else 0))
    assert mp.nchecksums == total
    assert mp.gather_ops() == ((2 * ngroups, False) if per_group else (2, True))
    layout, sb = hdfs.multi_layout(pk, gp, 1)
    host = np.zeros(int(sb[0]) + 16, np.uint8)
    for _, soff, poff, nbytes in layout.astype(np.int64):
        host[soff:soff + nbytes] = payload[poff:poff + nbytes]
    shard = torch.from_numpy(host).cuda()
    out = torch.full((total,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    mp.exec([shard.data_ptr()], out.data_ptr())
    m.sync()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    tmp = torch.cuda.Stream()
    out.fill_(0x5A5A5A5A)
    torch.cuda.synchronize()
    mp.exec([shard.data_ptr()], out.data_ptr(), [tmp])
    del tmp
    gc.collect()
    cs = torch.cuda.Stream()
    mp.exec([shard.data_ptr()], out.data_ptr(), [cs])  # (switch: an event on the freed-by-caller stream)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=cs, capture_error_mode="thread_local"):
        for _ in range(2):
            mp.exec([shard.data_ptr()], out.data_ptr(), [cs])
    for _ in range(2):
        out.fill_(0x5A5A5A5A)
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    del graph
    mp.close()
    m.close()


@pytest.mark.parametrize("self_send", [False, True, "packed"])
def test_multi_plan_pipelined(hdfs, orc, self_send):
    """CRC32C_MULTI_PIPELINE: consecutive execs overlap (two exec streams, two
    local arrays, the gather on the plan's comm stream); after
    crc32c_multi_plan_join every file's checksums are in its root array,
    bit-exact against the oracle -- host-issued over 4 rotating files and
    root arrays, into ONE root array (the in-place launches stay in exec
    order: the last file's checksums win), and captured into a graph with
    the join inside the capture, replayed twice.  With
    CRC32C_MULTI_SELF_SEND every exec's checksums also travel through the
    RCCL group on the comm stream; "packed": the groups' checksum ranges 37
    apart in the file, so the gather is packed (staging array + scatter
    kernel on the caller's stream)."""
    torch = _torch()
    gp, nfiles = 4, 4
    pk = oracle.uniform_packets(8 * gp)  # 8 blocks of 4 packets (2 MiB files)
    if self_send == "packed":
        pk["out_idx"] = np.array([(i // gp) * (gp * 128 + 37) + (i % gp) * 128 for i in range(pk.size)], np.uint64)
    flags = hdfs.CRC32C_MULTI_PIPELINE | (hdfs.CRC32C_MULTI_SELF_SEND if self_send else 0)
    m = hdfs.Multi([0])
    mp = m.plan(pk, gp, flags)
    assert mp.gather_ops() == ((2, True) if self_send == "packed" else (2 if self_send else 0, False))
    layout, sb = hdfs.multi_layout(pk, gp, 1)
    shards, wants = [], []
    for f in range(nfiles):
        payload = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 16, 900 + f)
        host = np.zeros(int(sb[0]) + 16, np.uint8)
        for _, soff, poff, nbytes in layout.astype(np.int64):
            host[soff:soff + nbytes] = payload[poff:poff + nbytes]
        shards.append(torch.from_numpy(host).cuda())
        wants.append(orc.batch(payload, pk, mp.nchecksums))
    outs = [torch.zeros(mp.nchecksums, dtype=torch.int32, device="cuda") for _ in range(nfiles)]
    cs = torch.cuda.Stream()
    torch.cuda.synchronize()

    def run(n, same=None):
        for k in range(n):
            f = k % nfiles
            mp.exec([shards[f].data_ptr()], (same if same is not None else outs[f]).data_ptr(), [cs])
        mp.join([cs])

    run(2 * nfiles + 1)
    cs.synchronize()
    for f in range(nfiles):
        assert np.array_equal(outs[f].cpu().numpy().view(np.uint32), wants[f]), f
    one = torch.zeros_like(outs[0])
    torch.cuda.synchronize()
    run(7, same=one)  # (files 0 1 2 3 0 1 2: the last is file 2)
    cs.synchronize()
    assert np.array_equal(one.cpu().numpy().view(np.uint32), wants[2])
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=cs, capture_error_mode="thread_local"):
        run(6)
    for _ in range(2):
        for o in outs:
            o.zero_()
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        for f in range(nfiles):
            assert np.array_equal(outs[f].cpu().numpy().view(np.uint32), wants[f]), f
    del graph
    mp.close()
    plain = m.plan(pk, gp, 0)
    plain.join([cs])  # (no pipeline: nothing to join)
    plain.close()
    m.close()


def test_multi_plan_refuses_too_many_gather_transfers(hdfs, orc):
    """Per group (CRC32C_MULTI_PER_GROUP_RECV), a gather of more than 4096
    point-to-point transfers in one RCCL group (here 4100 one-packet groups
    whose checksum ranges leave gaps, sent to self) is refused at plan
    creation with -E2BIG instead of being posted.  Packed (the default), the
    same plan posts one pair and its scatter kernel places all 4100 ranges:
    bit-exact, gaps untouched."""
    torch = _torch()
    pk = oracle.uniform_packets(4100, 512, 512)
    pk["out_idx"] = np.arange(4100, dtype=np.uint64) * 2  # (a gap after every group)
    m = hdfs.Multi([0])
    per_group = hdfs.CRC32C_MULTI_SELF_SEND | hdfs.CRC32C_MULTI_PER_GROUP_RECV
    try:
        with pytest.raises(hdfs.Crc32cError) as e:
            m.plan(pk, 1, per_group)
        assert e.value.rc == -7 and "group_packets" in str(e.value)  # -E2BIG
        m.plan(pk[:4000], 1, per_group).close()  # (4000 transfers: accepted)
        mp = m.plan(pk, 1, hdfs.CRC32C_MULTI_SELF_SEND)
        assert mp.gather_ops() == (2, True)
        payload = oracle.xorshift64_bytes(4100 * 512 + 16, 516)
        layout, sb = hdfs.multi_layout(pk, 1, 1)
        host = np.zeros(int(sb[0]) + 16, np.uint8)
        for _, soff, poff, nbytes in layout.astype(np.int64):
            host[soff:soff + nbytes] = payload[poff:poff + nbytes]
        shard = torch.from_numpy(host).cuda()
        out = torch.full((2 * 4100,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        mp.exec([shard.data_ptr()], out.data_ptr())
        m.sync()
        want = np.full(2 * 4100, 0x5A5A5A5A, np.uint32)
        want[0::2] = orc.batch(payload, pk, 2 * 4100)[0::2]
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
        mp.close()
    finally:
        m.close()


def test_multi_rank_mode_single_rank(hdfs, orc):
    """One-process-per-GPU communicator (ncclCommInitRank with an id from
    crc32c_multi_unique_id), nranks = 1: mixed-bpc blocks of ragged packets
    with empty last packets, gathered into place on rank 0."""
    torch = _torch()
    uid = hdfs.multi_unique_id()
    assert len(uid) == 128
    m = hdfs.Multi(device=0, rank=0, nranks=1, uid=uid)
    pk = oracle.mixed_packets(130)
    pk["bpc"][7::9] = 1536  # general tiles too
    pk["len"][63::64] = 0  # each block ends with the empty last packet
    pk["len"][5] = 1000
    per = (pk["len"].astype(np.int64) + pk["bpc"] - 1) // pk["bpc"]
    pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    payload = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 16, 31)
    mp = m.plan(pk, 64, hdfs.CRC32C_MULTI_SELF_SEND | hdfs.CRC32C_BIG_ENDIAN)
    layout, sb = hdfs.multi_layout(pk, 64, 1)
    host = np.zeros(int(sb[0]) + 16, np.uint8)
    for rank, soff, poff, nbytes in layout.astype(np.int64):
        host[soff:soff + nbytes] = payload[poff:poff + nbytes]
    shard = torch.from_numpy(host).cuda()
    out = torch.full((mp.nchecksums,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    mp.exec([shard.data_ptr()], out.data_ptr())
    m.sync()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), orc.batch(payload, pk, mp.nchecksums, big_endian=True))
    # successive execs on alternating streams (they reuse the plan's local
    # array: each waits for the previous one), two different shards
    torch_streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    host2 = host.copy()
    host2[:host2.size - 16] ^= 0x5C
    payload2 = payload.copy()
    for rank, soff, poff, nbytes in layout.astype(np.int64):
        payload2[poff:poff + nbytes] = host2[soff:soff + nbytes]
    shard2 = torch.from_numpy(host2).cuda()
    outs = [torch.zeros_like(out) for _ in range(6)]
    torch.cuda.synchronize()
    for k in range(6):
        mp.exec([(shard if k % 2 == 0 else shard2).data_ptr()], outs[k].data_ptr(), [torch_streams[k % 2].cuda_stream])
    torch.cuda.synchronize()
    want2 = orc.batch(payload2, pk, mp.nchecksums, big_endian=True)
    for k in range(6):
        assert np.array_equal(outs[k].cpu().numpy().view(np.uint32),
                              want2 if k % 2 else orc.batch(payload, pk, mp.nchecksums, big_endian=True)), k
    mp.close()
    m.close()


def test_multi_plan_refuses_a_device_twice(hdfs):
    """RCCL has one rank per GPU: a one-process multi handle listing a device
    twice can deal host batches (crc32c_multi_batch_host) but its plan is
    refused at creation, not at the first exec."""
    m = hdfs.Multi([0, 0])
    with pytest.raises(hdfs.Crc32cError) as e:
        m.plan(oracle.uniform_packets(128), 64)
    assert e.value.rc == -22 and "twice" in str(e.value)
    m.close()


def test_last_path_gpu(hdfs, orc):
    """crc32c_chunks reports the GPU path when it ran there (CRC32C_CPU_FALLBACK
    set or not)."""
    pkt = oracle.xorshift64_bytes(65536, 98)
    assert np.array_equal(hdfs.chunks(pkt, 512, hdfs.CRC32C_CPU_FALLBACK), orc.chunks(pkt, 512))
    assert hdfs.last_path() == hdfs.PATH_GPU


# ---- verification with a mismatch bitmap -----------------------------------------
def _bitmap_verify(plan, expected: np.ndarray, stream, payload=0):
    torch = _torch()
    n = expected.size
    exp = torch.from_numpy(expected.view(np.int32).copy()).cuda()
    res = torch.zeros(2, dtype=torch.int32, device="cuda")
    words = (n + 31) // 32
    bits = torch.full((max(words, 1),), -1, dtype=torch.int32, device="cuda")  # stale bits: must be cleared
    plan.verify(payload, exp.data_ptr(), res.data_ptr(), stream.cuda_stream, dev_bad_bits=bits.data_ptr())
    stream.synchronize()
    b = bits.cpu().numpy().view(np.uint32)[:words]
    flags = np.unpackbits(b.view(np.uint8), bitorder="little")
    assert not flags[n:].any()  # bits past the last checksum stay clear
    return res.cpu().numpy().view(np.uint32).tolist(), np.flatnonzero(flags[:n])


def test_verify_bitmap_every_item_kind(hdfs, gpu_ctx, orc):
    """crc32c_plan_verify_bitmap ("emit a mismatch
    bitmap"): the set of mismatching checksums equals the set corrupted --
    through power-of-two tiles, general tiles and items (bpc 1000, ragged
    tails), and a FUSE-shaped buffer-list write plan (chunks spanning buffers,
    zero-fill constants); corrupted payload bytes and expected values alike;
    count and lowest index agree with the bitmap; a clean run sets no bit."""
    torch = _torch()
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(818)
    pk = oracle.mixed_packets(48, bpcs=(512, 1000, 4096))
    pk["len"] = rng.integers(1, 65537, pk.size).astype(np.uint32)
    pk["len"][:24] = 65536
    per = (pk["len"].astype(np.uint64) + pk["bpc"] - 1) // pk["bpc"]
    pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    payload = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 64, 818)
    n = hdfs.total_checksums(pk)
    want = orc.batch(payload, pk, n)
    dev = torch.from_numpy(payload).cuda()
    plan = hdfs.Plan(gpu_ctx, pk)
    assert _bitmap_verify(plan, want, s, dev.data_ptr())[0] == [0, 0xFFFFFFFF]
    bad = set(int(x) for x in rng.choice(n, 40, replace=False))
    exp = want.copy()
    for i in sorted(bad)[::2]:
        exp[i] ^= np.uint32(1 << int(rng.integers(0, 32)))
    payload_bad = set(sorted(bad)[1::2])
    for i in sorted(payload_bad):  # the rest by a flipped payload byte inside that checksum's chunk
        p = int(np.searchsorted(pk["out_idx"], i, side="right") - 1)
        k = i - int(pk["out_idx"][p])
        lo = k * int(pk["bpc"][p])
        hi = min(lo + int(pk["bpc"][p]), int(pk["len"][p]))
        dev[int(pk["payload_off"][p]) + int(rng.integers(lo, hi))] ^= 0x40
    (cnt, first), idx = _bitmap_verify(plan, exp, s, dev.data_ptr())
    assert set(idx.tolist()) == bad and cnt == len(bad) and first == min(bad)
    # one bitmap reused by back-to-back verifies on two streams: the second
    # clears it only after the first (which sets other bits) has finished
    exp_a = torch.from_numpy(exp.view(np.int32).copy()).cuda()
    exp_b = torch.from_numpy(want.view(np.int32).copy()).cuda()
    exp_b[n - 1] ^= 1
    bits = torch.zeros((n + 31) // 32, dtype=torch.int32, device="cuda")
    res_a = torch.zeros(2, dtype=torch.int32, device="cuda")
    res_b = torch.zeros(2, dtype=torch.int32, device="cuda")
    s2 = torch.cuda.Stream()
    for _ in range(3):
        plan.verify(dev.data_ptr(), exp_a.data_ptr(), res_a.data_ptr(), s.cuda_stream, dev_bad_bits=bits.data_ptr())
        plan.verify(dev.data_ptr(), exp_b.data_ptr(), res_b.data_ptr(), s2.cuda_stream,
                    dev_bad_bits=bits.data_ptr())
        torch.cuda.synchronize()
        b = np.unpackbits(bits.cpu().numpy().view(np.uint8), bitorder="little")[:n]
        want_b = sorted(payload_bad | {n - 1})  # the payload is still corrupted
        assert np.flatnonzero(b).tolist() == want_b
        assert res_b.cpu().numpy().view(np.uint32).tolist() == [len(want_b), want_b[0]]
        assert res_a.cpu().numpy().view(np.uint32).tolist() == [len(bad), min(bad)]
    plan.close()
    # buffer-list write plan: TRUNCATE | NULLPADDING | THEDATA | TRAILINGDATA
    bufs, devs, stream_bytes = _fuse_write_buffers(torch, rng, [10000, 300000, 1 << 20, 77777],
                                                   [False, True, False, False], 900)
    length = stream_bytes.size - 11
    wplan = gpu_ctx.write_plan(bufs, 0, length, 0, 65536, 512)
    want = _expected_write(orc, stream_bytes, 0, length, 0, 65536, 512)
    assert _bitmap_verify(wplan, want, s)[0] == [0, 0xFFFFFFFF]
    bad = sorted(set(int(x) for x in rng.choice(want.size, 25, replace=False)) | {0, want.size - 1})
    exp = want.copy()
    exp[bad] ^= np.uint32(0x80000000)
    (cnt, first), idx = _bitmap_verify(wplan, exp, s)
    assert idx.tolist() == bad and cnt == len(bad) and first == 0
    wplan.close()


# ---- an fsx-style sequence of writes (the reference's only integration test) ----
def test_fsx_style_write_sequence(hdfs, gpu_ctx, orc):
    """README.md:35-39's manual test runs fsx against a MiniCluster so that
    writes span many blocks.  Here: 60 random file operations on a model
    file (appends, writes inside the last block, writes past EOF, writes
    into earlier blocks, ftruncate extensions and shrinks), each turned into
    hadoop_fuse_write's buffers (fuse.c:1348-1480: TRUNCATE, NULLPADDING,
    THEDATA, TRAILINGDATA) and hadoop_fuse_do_write's block writes
    (fuse.c:466-647: the block under construction from its offset, then new
    blocks from 0, bufferoffset advancing), every block write checksummed by
    one crc32c_plan_create_buffers plan over the device buffers and compared
    with the oracle over the bytes it sends.  256 KiB blocks, so writes span
    many of them."""
    torch = _torch()
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(0xF5)
    B, P = 256 << 10, 65536
    f = np.zeros(0, np.uint8)
    nwrites = 0
    for op in range(60):
        L = f.size
        kind = rng.choice(["append", "last_block", "past_eof", "earlier", "extend", "shrink"],
                          p=[0.3, 0.15, 0.15, 0.2, 0.1, 0.1])
        if kind == "shrink":
            f = f[:int(rng.integers(0, L + 1))]
            continue
        data = oracle.xorshift64_bytes(int(rng.integers(1, 700000)), 1000 + op)
        last = (L - 1) // B * B if L else 0
        if kind == "append":
            off = L
        elif kind == "last_block":
            off = int(rng.integers(last, L + 1))
        elif kind == "past_eof":
            off = L + int(rng.integers(1, 300000))
        elif kind == "earlier":
            off = int(rng.integers(0, max(last, 1)))
        else:  # ftruncate extension: a NULL buffer from EOF
            off, data = L, None
        parts = []  # (host bytes, is_null)
        if kind == "extend":
            parts.append((np.zeros(int(rng.integers(1, 900000)), np.uint8), True))
            start = L
        elif off < last:  # into an earlier block: keep its head, rewrite from there, re-append the tail
            start = off // B * B
            parts.append((f[start:off], False))
            parts.append((data, False))
            if off + data.size < L:
                parts.append((f[off + data.size:], False))
        else:
            start = min(off, L)
            if off > L:
                parts.append((np.zeros(off - L, np.uint8), True))
            parts.append((data, False))
        bufs, devs = [], []
        for host, is_null in parts:
            if is_null:
                bufs.append((0, host.size))
                continue
            skew = int(rng.integers(0, 16))
            t = torch.zeros(host.size + 32, dtype=torch.uint8, device="cuda")
            t[skew:skew + host.size].copy_(torch.from_numpy(np.ascontiguousarray(host)))
            devs.append(t)
            bufs.append((t.data_ptr() + skew, host.size))
        stream_bytes = np.concatenate([h for h, _ in parts]) if parts else np.zeros(0, np.uint8)
        # hadoop_fuse_do_write: the block under construction from its offset, then new blocks
        total, boff, pos = stream_bytes.size, start % B, 0
        while pos < total:
            n = min(B - boff, total - pos)
            plan = gpu_ctx.write_plan(bufs, pos, n, boff, P, 512)
            want = _expected_write(orc, stream_bytes, pos, n, boff, P, 512)
            assert plan.nchecksums == want.size, (op, kind, pos, n, boff)
            assert np.array_equal(_run_plan(plan, want.size, s), want), (op, kind, pos, n, boff)
            plan.close()
            nwrites += 1
            pos += n
            boff = 0
        f = np.concatenate([f[:start], stream_bytes])
    assert nwrites > 60


def test_plans_created_while_another_thread_captures(hdfs, gpu_ctx, orc):
    """Plan create / exec / destroy on one thread while another thread
    captures a graph in global mode (torch.cuda.graph's default): no
    device-wide synchronisation and no call that would invalidate the
    capture.  48 plans of growing shapes (new pool blocks, more than the old
    32-block epoch) are created, run on their own stream and destroyed during
    the capture; the captured launch replays exactly afterwards, and every
    plan's checksums are right."""
    import threading

    torch = _torch()
    payload = oracle.xorshift64_bytes(200 * 65536 + 16, 55)
    dpay = torch.from_numpy(payload).cuda()
    pk = oracle.uniform_packets(64)
    want = orc.batch(payload, pk, 8192)
    plan = gpu_ctx.plan(pk)
    out_g = torch.zeros(8192, dtype=torch.int32, device="cuda")
    plan.exec(dpay.data_ptr(), out_g.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    shapes = []
    for k in range(48):
        q = oracle.uniform_packets(1 + (k * 37) % 199, 65536, (512, 1536, 1024)[k % 3])
        q["len"][-1] -= 7 * k
        shapes.append(q)
    outs = [torch.zeros(max(oracle.total_checksums(q), 1), dtype=torch.int32, device="cuda") for q in shapes]
    side = torch.cuda.Stream()
    started, finished, errs = threading.Event(), threading.Event(), []

    def worker():
        started.wait(60)
        try:
            for q, o in zip(shapes, outs):
                p = gpu_ctx.plan(q)
                p.exec(dpay.data_ptr(), o.data_ptr(), side.cuda_stream)
                p.close()
        except Exception as e:  # noqa: BLE001
            errs.append(e)
        finished.set()

    t = threading.Thread(target=worker)
    t.start()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    try:
        with torch.cuda.graph(g, stream=cap):  # capture_error_mode="global"
            plan.exec(dpay.data_ptr(), out_g.data_ptr(), cap.cuda_stream)
            started.set()
            assert finished.wait(120)
    finally:
        started.set()
        t.join()
    assert not errs, errs
    out_g.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out_g.cpu().numpy().view(np.uint32), want)
    for q, o in zip(shapes, outs):
        n = oracle.total_checksums(q)
        assert np.array_equal(o.cpu().numpy().view(np.uint32)[:n], orc.batch(payload, q, n))
    del g
    plan.close()


def test_last_plan_of_a_closed_context_destroyed_during_a_capture(hdfs, orc):
    """a plan that outlives crc32c_ctx_destroy (a garbage
    collector freeing it late) is the context's last reference; destroying it
    must not tear the context down on the spot (stream synchronisation,
    hipFree) while another thread captures a graph in global mode.  The
    teardown is deferred to the next crc32c_ctx_create / _destroy: the
    capture stays valid and replays exactly; the deferred context is torn
    down by the next create."""
    import threading

    torch = _torch()
    payload = oracle.xorshift64_bytes(64 * 65536, 56)
    dpay = torch.from_numpy(payload).cuda()
    pk = oracle.uniform_packets(64)
    want = orc.batch(payload, pk, 8192)
    keep = hdfs.Context(0)  # (its plan is what the capture records)
    plan = keep.plan(pk)
    out_g = torch.zeros(8192, dtype=torch.int32, device="cuda")
    plan.exec(dpay.data_ptr(), out_g.data_ptr(), torch.cuda.current_stream())
    doomed_ctx = hdfs.Context(0)
    doomed = [doomed_ctx.plan(pk) for _ in range(3)]
    outs = [torch.zeros(8192, dtype=torch.int32, device="cuda") for _ in doomed]
    side = torch.cuda.Stream()
    for p_, o in zip(doomed, outs):
        p_.exec(dpay.data_ptr(), o.data_ptr(), side)
    torch.cuda.synchronize()
    doomed_ctx.close()  # (the plans hold it)
    started, finished, errs = threading.Event(), threading.Event(), []

    def worker():
        started.wait(60)
        try:
            for p_ in doomed:
                p_.close()  # (the last one drops the context's last reference)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
        finished.set()

    t = threading.Thread(target=worker)
    t.start()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    try:
        with torch.cuda.graph(g, stream=cap):  # capture_error_mode="global"
            plan.exec(dpay.data_ptr(), out_g.data_ptr(), cap.cuda_stream)
            started.set()
            assert finished.wait(120)
    finally:
        started.set()
        t.join()
    assert not errs, errs
    out_g.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out_g.cpu().numpy().view(np.uint32), want)
    for o in outs:
        assert np.array_equal(o.cpu().numpy().view(np.uint32), want)
    del g
    hdfs.Context(0).close()  # (a create tears the deferred context down)
    plan.close()
    keep.close()


# ---- many blocks of one shape in one launch (concurrent block writes) -------
def _block_shape(kind):
    if kind == "full":  # one 4 MiB block of 64 x 64 KiB packets
        return oracle.uniform_packets(64)
    if kind == "ragged":  # a short block: 15 packets + a 1000-byte tail packet (general tile)
        pk = oracle.uniform_packets(16)
        pk["len"][-1] = 1000
        return pk
    if kind == "bpc1536":
        return oracle.uniform_packets(8, 65536, 1536)
    if kind == "tiny_tail":  # a 2-byte tail: no multi-block form, one launch per block
        pk = oracle.uniform_packets(4)
        pk["len"][-1] = 65536 - 510
        return pk
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["full", "ragged", "bpc1536", "tiny_tail"])
def test_plan_exec_blocks(hdfs, gpu_ctx, orc, kind):
    """crc32c_plan_exec_blocks: one block's plan run over 40 blocks in
    separate device buffers (some off 16-byte alignment, outputs in separate
    arrays and inside one shared array) -- two launches of <= 32 blocks --
    every block bit-exact against the oracle."""
    torch = _torch()
    pk = _block_shape(kind)
    n = oracle.total_checksums(pk)
    ext = int((pk["payload_off"] + pk["len"]).max())
    bufs, pays, outs, wants = [], [], [], []
    shared = torch.zeros(20 * n + 8, dtype=torch.int32, device="cuda")
    for b in range(40):
        skew = (b * 5) % 16 if b % 3 == 0 else 0
        host = oracle.xorshift64_bytes(ext + 32, 900 + b)
        t = torch.from_numpy(host).cuda()
        bufs.append(t)
        pays.append(t.data_ptr() + skew)
        wants.append(orc.batch(host[skew:], pk, n))
        if b % 2:
            o = torch.full((n,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
            bufs.append(o)
            outs.append((o, 0))
        else:
            outs.append((shared, (b // 2) * n))
    plan = gpu_ctx.plan(pk)
    stream = torch.cuda.current_stream()
    plan.exec_blocks(pays, [o.data_ptr() + 4 * off for o, off in outs], stream.cuda_stream)
    torch.cuda.synchronize()
    for b, (o, off) in enumerate(outs):
        got = o.cpu().numpy().view(np.uint32)[off:off + n]
        assert np.array_equal(got, wants[b]), (kind, b)
    plan.close()


def test_block_queue_threads(hdfs, gpu_ctx, orc):
    """crc32c_blocks: 12 threads, each writing 6 blocks of 4 MiB one after
    another through crc32c_block_checksums (no batching by the caller): every
    block bit-exact against the oracle, and the queue carried them in far
    fewer launches than blocks (group commit)."""
    import threading

    torch = _torch()
    pk = _block_shape("full")
    n = oracle.total_checksums(pk)
    nthreads, per = 12, 6
    hosts = [oracle.xorshift64_bytes(64 * 65536, 7000 + k) for k in range(nthreads * per)]
    devs = [torch.from_numpy(h).cuda() for h in hosts]
    outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in hosts]
    torch.cuda.synchronize()
    plan = gpu_ctx.plan(pk)
    q = plan.blocks(max_blocks=12, window_us=200)
    errs = []
    go = threading.Barrier(nthreads)

    def worker(k):
        try:
            go.wait()
            for j in range(per):
                i = k * per + j
                q.checksums(devs[i].data_ptr(), outs[i].data_ptr())
                # the checksums are in device memory now: check this block right away
                assert np.array_equal(outs[i].cpu().numpy().view(np.uint32), orc.batch(hosts[i], pk, n)), i
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs[:3]
    flushes, blocks = q.stats()
    assert blocks == nthreads * per and flushes < blocks // 2, (flushes, blocks)
    # explicit submit / flush / wait
    for i in range(5):
        outs[i].zero_()
    torch.cuda.synchronize()
    tickets = [q.submit(devs[i].data_ptr(), outs[i].data_ptr()) for i in range(5)]
    q.flush()
    for t in reversed(tickets):
        q.wait(t)
    for i in range(5):
        assert np.array_equal(outs[i].cpu().numpy().view(np.uint32), orc.batch(hosts[i], pk, n))
    with pytest.raises(hdfs.Crc32cError):
        q.wait(10**9)
    # a partial batch goes out when its window has passed (no flush call)
    for i in range(3):
        outs[i].zero_()
    torch.cuda.synchronize()
    tickets = [q.submit(devs[i].data_ptr(), outs[i].data_ptr()) for i in range(3)]
    q.wait(tickets[-1])
    for i in range(3):
        assert np.array_equal(outs[i].cpu().numpy().view(np.uint32), orc.batch(hosts[i], pk, n))
    # destroy launches what is still queued and waits for it
    for i in range(2):
        outs[i].zero_()
    torch.cuda.synchronize()
    q2 = plan.blocks(max_blocks=12, window_us=10**6)
    for i in range(2):
        q2.submit(devs[i].data_ptr(), outs[i].data_ptr())
    q2.close()
    for i in range(2):
        assert np.array_equal(outs[i].cpu().numpy().view(np.uint32), orc.batch(hosts[i], pk, n))
    q.close()
    plan.close()


def test_block_queue_failed_flush_is_its_own(hdfs, gpu_ctx, orc):
    """A flush whose issue fails (crc32c_debug_blocks_fail_flushes) fails
    exactly its own tickets: the flush before it and every flush after it
    succeed, bit-exact (one sticky queue error failed every later
    write); and a submit after destroy began is refused, never queued."""
    torch = _torch()
    pk = _block_shape("full")
    n = oracle.total_checksums(pk)
    hosts = [oracle.xorshift64_bytes(64 * 65536, 9500 + k) for k in range(10)]
    want = [orc.batch(h, pk, n) for h in hosts]
    devs = [torch.from_numpy(h).cuda() for h in hosts]
    outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in hosts]
    torch.cuda.synchronize()
    plan = gpu_ctx.plan(pk)
    q = plan.blocks(max_blocks=4, window_us=10**6)
    first = [q.submit(devs[i].data_ptr(), outs[i].data_ptr()) for i in range(4)]  # one full flush
    for t in first:
        q.wait(t)
    q.debug_fail_flushes(1)
    bad = [q.submit(devs[i].data_ptr(), outs[i].data_ptr()) for i in (4, 5)]
    q.flush()
    for t in bad:
        with pytest.raises(hdfs.Crc32cError) as ei:
            q.wait(t)
        assert ei.value.rc == -5  # -EIO
    later = [q.submit(devs[i].data_ptr(), outs[i].data_ptr()) for i in range(6, 10)]
    for t in later + first:
        q.wait(t)
    for i in list(range(4)) + list(range(6, 10)):
        assert np.array_equal(outs[i].cpu().numpy().view(np.uint32), want[i]), i
    for i in (4, 5):  # nothing was launched for the failed flush
        assert not outs[i].cpu().numpy().any()
    assert q.stats() == (3, 10)
    q.close()
    plan.close()


@pytest.mark.parametrize("shape", ["12", "16x15"])
def test_resident_kernel_blocks(hdfs, gpu_ctx, orc, shape, monkeypatch):
    """The debug library's resident kernel (A/B experiment, DESIGN.md section
    6): blocks submitted from 8 threads, 2 in flight each, bit-exact; the
    kernel exits after idle_us with nothing queued and a later submit
    relaunches it; destroy with blocks still queued returns (the kernel
    exits on the stop word) and a plain launch runs after it.  Every wave of
    the kernel has its own bounded wait, so nothing here can hang the GPU."""
    import threading
    import time

    torch = _torch()
    pk = _block_shape("full")
    n = oracle.total_checksums(pk)
    hosts = [oracle.xorshift64_bytes(64 * 65536, 8800 + k) for k in range(16)]
    want = [orc.batch(h, pk, n) for h in hosts]
    devs = [torch.from_numpy(h).cuda() for h in hosts]
    outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in hosts]
    torch.cuda.synchronize()
    plan = gpu_ctx.plan(pk)
    monkeypatch.setenv("HDFS_CRC32C_RESIDENT_WAVES", shape)  # (read at create: the kernel's shape)
    r = hdfs.Resident(plan, idle_us=500)
    errs = []

    def worker(k):
        try:
            ring = []
            for i in range(20):
                b = 2 * k + (i % 2)
                if len(ring) == 2:
                    t, bb = ring.pop(0)
                    r.wait(t)
                    got = outs[bb].cpu().numpy().view(np.uint32)
                    assert np.array_equal(got, want[bb]), (k, i)
                    outs[bb].zero_()
                    torch.cuda.synchronize()
                ring.append((r.submit(devs[b].data_ptr(), outs[b].data_ptr()), b))
            for t, bb in ring:
                r.wait(t)
                assert np.array_equal(outs[bb].cpu().numpy().view(np.uint32), want[bb]), k
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs[:3]
    first = r.launches()
    time.sleep(0.05)  # past idle_us: the kernel has exited
    outs[0].zero_()
    torch.cuda.synchronize()
    r.wait(r.submit(devs[0].data_ptr(), outs[0].data_ptr()))
    assert np.array_equal(outs[0].cpu().numpy().view(np.uint32), want[0])
    assert r.launches() > first
    for i in range(10):  # destroy with blocks queued
        r.submit(devs[i].data_ptr(), outs[i].data_ptr())
    r.close()
    outs[1].zero_()
    plan.exec(devs[1].data_ptr(), outs[1].data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(outs[1].cpu().numpy().view(np.uint32), want[1])
    plan.close()


def test_block_queue_resident_mode(hdfs, gpu_ctx, orc):
    """crc32c_blocks_create_resident -- the PRODUCT library's resident-kernel
    mode of the block queue (opt-in): 16 writer threads, 2 blocks in flight
    each through the queue calls (crc32c_block_submit / _wait, and
    crc32c_block_checksums), every block bit-exact against the oracle; the
    kernel exits idle_us after the last block and the next submit relaunches
    it; flush is a no-op; a misaligned output and a plan of half tiles
    (bpc 700) are refused; destroy with blocks queued completes them, refuses later
    submits, and a plain launch runs after it.  Every wave of the kernel has
    a bounded wait, so nothing here can hang the GPU."""
    import threading
    import time

    torch = _torch()
    pk = _block_shape("full")
    n = oracle.total_checksums(pk)
    nthreads, per, depth = 16, 24, 2
    hosts = [oracle.xorshift64_bytes(64 * 65536, 8300 + k) for k in range(nthreads * depth)]
    want = [orc.batch(h, pk, n) for h in hosts]
    devs = [torch.from_numpy(h).cuda() for h in hosts]
    outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in hosts]
    torch.cuda.synchronize()
    plan = gpu_ctx.plan(pk)
    q = plan.blocks(resident=True, idle_us=500)
    errs = []
    go = threading.Barrier(nthreads)

    # (outputs are cleared by host-to-device copies, which need no CU: while
    # the resident kernel runs it holds every CU, and a fill kernel would
    # wait for its idle exit)
    zeros = torch.zeros(n, dtype=torch.int32).pin_memory()

    def worker(k):
        try:
            s = torch.cuda.Stream()
            ring = [None] * depth
            go.wait()
            for i in range(per + depth):
                slot = i % depth
                b = k * depth + slot
                if ring[slot] is not None:
                    q.wait(ring[slot])
                    assert np.array_equal(outs[b].cpu().numpy().view(np.uint32), want[b]), (k, i)
                if i < per:
                    with torch.cuda.stream(s):
                        outs[b].copy_(zeros, non_blocking=True)
                    s.synchronize()
                    ring[slot] = q.submit(devs[b].data_ptr(), outs[b].data_ptr())
                else:
                    ring[slot] = None
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs[:3]
    launches, blocks = q.stats()
    assert blocks == nthreads * per and 1 <= launches < blocks // 8, (launches, blocks)
    # idle exit, then a relaunch on the next block (crc32c_block_checksums = submit + wait)
    time.sleep(0.05)
    outs[0].zero_()
    torch.cuda.synchronize()
    q.flush()
    q.checksums(devs[0].data_ptr(), outs[0].data_ptr())
    assert np.array_equal(outs[0].cpu().numpy().view(np.uint32), want[0])
    assert q.stats()[0] > launches
    with pytest.raises(hdfs.Crc32cError) as ei:  # (payloads at any alignment; outputs 4-byte aligned)
        q.submit(devs[0].data_ptr(), outs[0].data_ptr() + 2)
    assert ei.value.rc == -22
    with pytest.raises(hdfs.Crc32cError):
        q.wait(10**9)
    # destroy with blocks queued: every one of them completes
    for i in range(10):
        outs[i].zero_()
    torch.cuda.synchronize()
    for i in range(10):
        q.submit(devs[i].data_ptr(), outs[i].data_ptr())
    q.close()
    for i in range(10):
        assert np.array_equal(outs[i].cpu().numpy().view(np.uint32), want[i]), i
    outs[1].zero_()
    plan.exec(devs[1].data_ptr(), outs[1].data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert np.array_equal(outs[1].cpu().numpy().view(np.uint32), want[1])
    plan.close()
    gplan = gpu_ctx.plan(oracle.uniform_packets(8, 65536, 700))  # (half tiles: their own kernel builds)
    with pytest.raises(hdfs.Crc32cError) as ei:
        gplan.blocks(resident=True)
    assert ei.value.rc == -22 and "half" in str(ei.value)
    gplan.close()


def test_block_queue_ring_reuse_two_in_flight(hdfs, gpu_ctx, orc):
    """crc32c_blocks with more tickets than its ring has slots (1024): 16
    threads keep two blocks in flight each (submit the next, then wait for
    the oldest), 80 blocks per thread = 1280 tickets, max_blocks 8 (launches
    capped at two in flight, the rest waiting in the ring).  Every output is
    zeroed before its block is submitted and checked right after its wait,
    so a launch that carried a stale ring slot or completed out of order
    shows."""
    import threading

    torch = _torch()
    pk = _block_shape("full")
    n = oracle.total_checksums(pk)
    nthreads, per, depth = 16, 80, 2
    hosts = [oracle.xorshift64_bytes(64 * 65536, 9100 + k) for k in range(nthreads * depth)]
    want = [orc.batch(h, pk, n) for h in hosts]
    devs = [torch.from_numpy(h).cuda() for h in hosts]
    outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in hosts]
    torch.cuda.synchronize()
    plan = gpu_ctx.plan(pk)
    q = plan.blocks(max_blocks=8, window_us=50)
    errs = []
    go = threading.Barrier(nthreads)

    def worker(k):
        try:
            s = torch.cuda.Stream()
            ring = [None] * depth
            go.wait()
            for i in range(per + depth):
                slot = i % depth
                b = k * depth + slot
                if ring[slot] is not None:
                    q.wait(ring[slot])
                    got = outs[b].cpu().numpy().view(np.uint32)
                    assert np.array_equal(got, want[b]), (k, i)
                if i < per:
                    with torch.cuda.stream(s):
                        outs[b].zero_()
                    s.synchronize()
                    ring[slot] = q.submit(devs[b].data_ptr(), outs[b].data_ptr())
                else:
                    ring[slot] = None
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs[:3]
    flushes, blocks = q.stats()
    assert blocks == nthreads * per and flushes <= blocks, (flushes, blocks)
    q.close()
    plan.close()


def test_verify_overlapping_launches_terminate(hdfs, gpu_ctx, orc):
    """The one verify overlap the library cannot order: a graph of captured
    verify launches replayed on one stream while the same plan is verified
    directly on another (a mismatching workgroup then waited for
    its launch's key forever).  With mismatches in every launch, both streams
    must finish (the key wait is bounded); every result is either exact or
    flagged CRC32C_VERIFY_OVERLAP; a verify after both is exact again."""
    torch = _torch()
    pk = oracle.uniform_packets(1024)
    n = oracle.total_checksums(pk)
    payload = oracle.xorshift64_bytes(int(pk["payload_off"][-1] + pk["len"][-1]) + 16, 4242)
    want = orc.batch(payload, pk, n)
    dpay = torch.from_numpy(payload).cuda()
    bad_idx = np.arange(5, n, n // 97)  # mismatches spread over most workgroups
    badv = want.copy()
    badv[bad_idx] ^= 0x0F0F
    bad = torch.from_numpy(badv.view(np.int32)).cuda()
    expect = (len(bad_idx), int(bad_idx.min()))
    plan = gpu_ctx.plan(pk)
    cap, direct = torch.cuda.Stream(), torch.cuda.Stream()
    nl = 6
    gres = [torch.zeros(2, dtype=torch.int32, device="cuda") for _ in range(nl)]
    dres = [torch.zeros(2, dtype=torch.int32, device="cuda") for _ in range(nl)]
    plan.verify(dpay.data_ptr(), bad.data_ptr(), gres[0].data_ptr(), cap.cuda_stream)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        for r in gres:
            plan.verify(dpay.data_ptr(), bad.data_ptr(), r.data_ptr(), cap.cuda_stream)
    torch.cuda.synchronize()
    replay = torch.cuda.Stream()
    with torch.cuda.stream(replay):
        g.replay()  # (not on the capture stream: the plan's ordering cannot see it)
    for r in dres:
        plan.verify(dpay.data_ptr(), bad.data_ptr(), r.data_ptr(), direct.cuda_stream)
    torch.cuda.synchronize()
    flagged = 0
    for r in gres + dres:
        c, first = (int(x) for x in r.cpu().numpy().view(np.uint32))
        if c & hdfs.CRC32C_VERIFY_OVERLAP:
            flagged += 1
        else:
            assert (c, first) == expect
    print("overlap-flagged results: %d of %d" % (flagged, 2 * nl))
    res = torch.zeros(2, dtype=torch.int32, device="cuda")
    plan.verify(dpay.data_ptr(), bad.data_ptr(), res.data_ptr(), direct.cuda_stream)
    torch.cuda.synchronize()
    assert tuple(int(x) for x in res.cpu().numpy().view(np.uint32)) == expect
    del g
    plan.close()


@pytest.mark.parametrize("npk", [64, 4096])
def test_verify_result_per_launch_graph_replays(hdfs, gpu_ctx, orc, npk):
    """Verification results are per launch, with no host reset: workgroup 0
    initialises the result and stores the launch's key (dispatch packet
    address + dispatch id), and only mismatching workgroups add after it.
    Back-to-back launches into the SAME result buffer, alternating clean and
    corrupt expected arrays, must each report their own counts (never a
    sum); a captured graph of [corrupt, clean, corrupt] launches replayed
    three times must leave each launch's own result after every replay (a
    replay reuses the captured kernel arguments, so only a device-side key
    tells its launches apart).  One 4 MiB block (256 workgroups) and config
    2 (one per CU)."""
    torch = _torch()
    pk = oracle.uniform_packets(npk)
    n = oracle.total_checksums(pk)
    payload = oracle.xorshift64_bytes(int(pk["payload_off"][-1] + pk["len"][-1]) + 16, 777 + npk)
    want = orc.batch(payload, pk, n)
    dpay = torch.from_numpy(payload).cuda()
    good = torch.from_numpy(want.view(np.int32).copy()).cuda()
    bad_idx = np.array([3, n // 2, n - 1, n // 3 + 7])
    badv = want.copy()
    badv[bad_idx] ^= 0x5A5A
    bad = torch.from_numpy(badv.view(np.int32)).cuda()
    plan = gpu_ctx.plan(pk)
    s = torch.cuda.Stream()
    res = torch.full((2,), 12345, dtype=torch.int32, device="cuda")
    expect_bad = (len(bad_idx), int(bad_idx.min()))
    for k in range(6):
        exp = bad if k % 2 else good
        plan.verify(dpay.data_ptr(), exp.data_ptr(), res.data_ptr(), s.cuda_stream)
        s.synchronize()
        r = tuple(int(x) for x in res.cpu().numpy().view(np.uint32))
        assert r == (expect_bad if k % 2 else (0, 0xFFFFFFFF)), (k, r)
    results = [torch.full((2,), 777, dtype=torch.int32, device="cuda") for _ in range(3)]
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for exp, r in zip((bad, good, bad), results):
            plan.verify(dpay.data_ptr(), exp.data_ptr(), r.data_ptr(), s.cuda_stream)
    for rep in range(3):
        g.replay()
        torch.cuda.synchronize()
        got = [tuple(int(x) for x in r.cpu().numpy().view(np.uint32)) for r in results]
        assert got == [expect_bad, (0, 0xFFFFFFFF), expect_bad], (rep, got)
    del g
    plan.close()


def _append_packets(length, blockoffset, bpc=512):
    """One block write of hadoop_rpc_send_packets(len = length, blockoffset)
    (hadooprpc.c:815-860: the first packet trimmed to a chunk boundary), its
    packets back to back from the block's payload start."""
    lens = _hdfs_mod().packetize(length, blockoffset, 65536, bpc)
    pk = np.zeros(len(lens), oracle.PACKET_DTYPE)
    off = oi = 0
    for i, ln in enumerate(lens):
        pk[i]["payload_off"], pk[i]["len"], pk[i]["bpc"], pk[i]["out_idx"] = off, ln, bpc, oi
        off += ln
        oi += -(-ln // bpc)
    return pk


def _hdfs_mod():
    from conftest import load_package

    return load_package()


# The shapes a FUSE daemon's block writes take (src/fuse.c:466-650): whole 4
# MiB blocks (the queue's plan) and the first block of an append at an
# unaligned offset (updateBlockForPipeline + write_block at blockoffset > 0),
# some ending mid-chunk (a write that is not a multiple of 512 bytes).
_APPENDS = [(4 * 2**20 - 100, 100), (4 * 2**20 - 4296, 4296), (4 * 2**20 - 196615, 196615),
            (1234567, 333), (65536 * 3 + 17, 0), (700, 4000)]


@pytest.mark.parametrize("resident", [True, False])
def test_block_queue_mixed_block_shapes(hdfs, gpu_ctx, orc, resident):
    """crc32c_block_submit_plan: 16 writer threads, 2 blocks in flight each,
    alternating whole blocks (the queue's plan) with unaligned appends of
    _APPENDS (their own plans: a trimmed first packet = a GenItem, tiles off
    16-byte alignment from it on, tails as general tiles / GenItems) and,
    through the group-commit queue, a bpc-1536 block (general tiles), the
    payloads at skews 0..15 -- through the resident kernel and through the
    group-commit queue; every block bit-exact against the oracle.  The
    resident queue starts in its aligned-only build and hands over to the
    general build at the first block that needs it; it refuses a plan of
    another checksum type and one of bpc 1536."""
    import threading

    torch = _torch()
    full = oracle.uniform_packets(64)
    # (+ through the group-commit queue, a block of bpc 1536: general tiles
    # of 3-block chunks, which the resident kernel refuses)
    shapes = [full] + [_append_packets(ln, off) for ln, off in _APPENDS]
    if not resident:
        shapes.append(oracle.uniform_packets(48, 65536, 1536))
    plans = [gpu_ctx.plan(pk) for pk in shapes]
    nthreads, per, depth = 16, 12, 2
    jobs = []  # (shape index, skew, host bytes)
    for k in range(nthreads * depth):
        si = 0 if k % 2 == 0 else 1 + (k // 2) % (len(shapes) - 1)
        ext = int((shapes[si]["payload_off"] + shapes[si]["len"]).max())
        jobs.append((si, (k * 7) % 16, oracle.xorshift64_bytes(ext + 32, 4400 + k)))
    want = [orc.batch(h[sk:], shapes[si], oracle.total_checksums(shapes[si])) for si, sk, h in jobs]
    devs = [torch.from_numpy(h).cuda() for _, _, h in jobs]
    outs = [torch.zeros(max(len(w), 1), dtype=torch.int32, device="cuda") for w in want]
    torch.cuda.synchronize()
    q = plans[0].blocks(resident=resident, idle_us=500, max_blocks=8, window_us=20)
    zeros = torch.zeros(max(o.numel() for o in outs), dtype=torch.int32).pin_memory()
    errs = []
    go = threading.Barrier(nthreads)

    def worker(k):
        try:
            s = torch.cuda.Stream()
            ring = [None] * depth
            go.wait()
            for i in range(per + depth):
                slot = i % depth
                b = k * depth + slot
                si, sk, _ = jobs[b]
                if ring[slot] is not None:
                    q.wait(ring[slot])
                    assert np.array_equal(outs[b].cpu().numpy().view(np.uint32)[:len(want[b])], want[b]), (k, i, si)
                if i < per:
                    with torch.cuda.stream(s):
                        outs[b].copy_(zeros[:outs[b].numel()], non_blocking=True)
                    s.synchronize()
                    ring[slot] = q.submit(devs[b].data_ptr() + sk, outs[b].data_ptr(), plan=plans[si] if si else None)
                else:
                    ring[slot] = None
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs[:3]
    if resident:
        crc32_plan = gpu_ctx.plan(shapes[1], hdfs.CRC32C_TYPE_CRC32)
        b1536 = gpu_ctx.plan(oracle.uniform_packets(48, 65536, 1536))
        for pl in (crc32_plan, b1536):
            with pytest.raises(hdfs.Crc32cError) as ei:
                q.submit(devs[1].data_ptr(), outs[1].data_ptr(), plan=pl)
            assert ei.value.rc == -22
        launches, blocks = q.stats()
        assert blocks == nthreads * per and launches >= 1
    q.close()
    if resident:
        crc32_plan.close()
        b1536.close()
    for pl in plans:
        pl.close()


def test_block_queue_resident_failed_slot_wait_takes_no_ticket(hdfs, gpu_ctx, orc):
    """a submit whose ring slot is still busy waits for it BEFORE
    taking a ticket, so a wait that gives up leaves no hole in the ticket
    sequence.  With the kernel held back (debug hook) 64 submits fill the
    ring; the 65th's slot wait is made to fail: -ETIMEDOUT, no ticket taken.
    Released, the same submit then gets ticket 64 and all 65 blocks complete
    bit-exact -- the queue was not wedged."""
    torch = _torch()
    pk = oracle.uniform_packets(8)
    n = oracle.total_checksums(pk)
    host = oracle.xorshift64_bytes(8 * 65536, 4242)
    want = orc.batch(host, pk, n)
    dev = torch.from_numpy(host).cuda()
    outs = torch.zeros((65, n), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    plan = gpu_ctx.plan(pk)
    q = plan.blocks(resident=True, idle_us=500)
    q.debug_resident_inject(True, 1)
    tickets = [q.submit(dev.data_ptr(), outs[i].data_ptr()) for i in range(64)]
    assert tickets == list(range(64)) and q.stats() == (0, 64)
    with pytest.raises(hdfs.Crc32cError) as ei:
        q.submit(dev.data_ptr(), outs[64].data_ptr())
    assert ei.value.rc == -110  # -ETIMEDOUT
    assert q.stats() == (0, 64)  # (no ticket was taken)
    q.debug_resident_inject(False, 0)
    assert q.submit(dev.data_ptr(), outs[64].data_ptr()) == 64
    for t in tickets + [64]:
        q.wait(t)
    got = outs.cpu().numpy().view(np.uint32)
    for i in range(65):
        assert np.array_equal(got[i], want), i
    q.close()
    plan.close()


def test_block_queue_resident_hands_over_to_general_build(hdfs, gpu_ctx, orc):
    """The resident queue runs its own plan's aligned blocks in the
    aligned-only kernel build; the first block that needs more -- here the
    same plan's block at a misaligned payload -- ends that launch at the
    block (its forwarder stops there) and starts the general build, which
    then serves every block: blocks before and after the hand-over bit-exact,
    two launches in all."""
    torch = _torch()
    pk = oracle.uniform_packets(16)
    n = oracle.total_checksums(pk)
    host = oracle.xorshift64_bytes(16 * 65536 + 32, 5150)
    dev = torch.from_numpy(host).cuda()
    outs = torch.zeros((12, n), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    plan = gpu_ctx.plan(pk)
    q = plan.blocks(resident=True, idle_us=200000)  # (the aligned-only launch is still running at the hand-over)
    skews = [0, 0, 0, 0, 5, 0, 0, 13, 0, 16, 3, 0]
    tickets = []
    for i, sk in enumerate(skews):
        tickets.append(q.submit(dev.data_ptr() + sk, outs[i].data_ptr()))
        if i == 3:
            for t in tickets:
                q.wait(t)
            assert q.stats() == (1, 4)
    for t in tickets:
        q.wait(t)
    assert q.stats() == (2, 12)
    got = outs.cpu().numpy().view(np.uint32)
    for i, sk in enumerate(skews):
        assert np.array_equal(got[i], orc.batch(host[sk:], pk, n)), i
    q.close()
    plan.close()


def test_verify_bitmap_more_mismatches_than_a_workgroup_lists(hdfs, gpu_ctx, orc):
    """a workgroup keeps its first 256 mismatching indices in LDS
    until it sees its launch's key; the ones past the list wait for the key
    per lane and set their bits directly.  A 64 MiB batch (32 tiles = 512
    checksums per workgroup) verified against expected values that are ALL
    wrong: every workgroup goes past its list.  The count, the lowest index
    and the bitmap name every checksum, and no overlap bit is set (nothing
    else runs)."""
    torch = _torch()
    s = torch.cuda.current_stream()
    pk = oracle.uniform_packets(1024)
    n = hdfs.total_checksums(pk)
    payload = oracle.xorshift64_bytes(1024 * 65536, 2026)
    want = orc.batch(payload, pk, n)
    dev = torch.from_numpy(payload).cuda()
    plan = hdfs.Plan(gpu_ctx, pk)
    res, bad = _bitmap_verify(plan, ~want, s, dev.data_ptr())
    assert res == [n, 0] and bad.size == n
    res, bad = _bitmap_verify(plan, want, s, dev.data_ptr())  # (and clean again right after)
    assert res == [0, 0xFFFFFFFF] and bad.size == 0
    plan.close()
