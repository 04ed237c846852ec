"""Parity of the HIP path with the oracle and the reference's golden vectors.

Every test calls the GPU through the C ABI (libhdfs_crc32c.so via ctypes);
torch only allocates device memory and provides the stream.  The bar is
bit-exact equality (integer work)."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import oracle
from conftest import golden_batch_packets, golden_fill

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch


def run_dev(hdfs, ctx, payload: np.ndarray, pk: np.ndarray, flags: int = 0, offset: int = 0) -> np.ndarray:
    """Device-resident plan execution; `offset` shifts the payload inside the
    device buffer (the plan itself sees payload_off values)."""
    torch = _torch()
    dev = torch.zeros(payload.size + offset + 64, dtype=torch.uint8, device="cuda")
    dev[offset:offset + payload.size].copy_(torch.from_numpy(payload))
    n = hdfs.total_checksums(pk)
    out = torch.full((max(n, 1),), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    plan = hdfs.Plan(ctx, pk, flags)
    assert plan.nchecksums == n
    stream = torch.cuda.current_stream()
    plan.exec(dev.data_ptr() + offset, out.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    plan.close()
    return out.cpu().numpy().view(np.uint32)[:n]


@pytest.mark.parametrize("name", ["c1_one_packet", "c3_one_block_4MiB", "c5_mixed_bpc_96", "ragged_tail_257",
                                  "c2_4096_packets", "c5_mixed_bpc_4096", "c4_file_128MiB", "c2_bpc1536"])
def test_golden_batches_device_resident(hdfs, gpu_ctx, golden, name):
    spec = [b for b in golden["batches"] if b["name"] == name][0]
    pk = golden_batch_packets(spec)
    payload = oracle.xorshift64_bytes(spec["payload_bytes"], spec["seed"])
    got = run_dev(hdfs, gpu_ctx, payload, pk)
    assert got.size == spec["nchecksums"]
    assert ["%08x" % v for v in got[:8]] == spec["head"]
    assert ["%08x" % v for v in got[-8:]] == spec["tail"]
    assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == spec["sha256_le"]


def test_golden_packets_host_path(hdfs, gpu_ctx, golden):
    for c in golden["packets"]["cases"]:
        buf = golden_fill(c["kind"], c["len"] + c["skip"], c["seed"])[c["skip"]:]
        pk = np.zeros(1, hdfs.PACKET_DTYPE)
        pk["len"] = c["len"]
        pk["bpc"] = c["bpc"]
        got = gpu_ctx.batch_host(np.ascontiguousarray(buf), pk)
        assert ["%08x" % v for v in got] == c["crcs"], (c["bpc"], c["kind"], c["len"])


def test_golden_packets_device_unaligned(hdfs, gpu_ctx, golden):
    # Every fixture packet placed at a 16-byte-misaligned device offset (the
    # general path) and at an aligned one (fast path where bpc allows).
    cases = golden["packets"]["cases"]
    bufs, pk = [], np.zeros(len(cases) * 2, hdfs.PACKET_DTYPE)
    off, out = 0, 0
    for i, c in enumerate(cases * 2):
        mis = 3 if i < len(cases) else 0
        buf = golden_fill(c["kind"], c["len"] + c["skip"], c["seed"])[c["skip"]:]
        off += mis
        pk[i] = (off, out, c["len"], c["bpc"])
        bufs.append((off, buf))
        off = (off + c["len"] + 15) & ~15
        out += (c["len"] + c["bpc"] - 1) // c["bpc"]
    payload = np.zeros(off + 16, np.uint8)
    for o, b in bufs:
        payload[o:o + b.size] = b
    got = run_dev(hdfs, gpu_ctx, payload, pk)
    want = [v for c in cases * 2 for v in c["crcs"]]
    assert ["%08x" % v for v in got] == want


def test_big_endian_flag(hdfs, gpu_ctx, orc):
    pk = oracle.mixed_packets(6, pkt_len=10000)
    payload = oracle.xorshift64_bytes(60000, 8)
    le = run_dev(hdfs, gpu_ctx, payload, pk)
    be = run_dev(hdfs, gpu_ctx, payload, pk, flags=hdfs.CRC32C_BIG_ENDIAN)
    assert np.array_equal(le, orc.batch(payload, pk, le.size))
    assert np.array_equal(be, le.byteswap())


def test_edge_cases(hdfs, gpu_ctx, orc):
    rows = [  # (len, bpc)
        (0, 512), (1, 512), (3, 512), (4, 512), (15, 512), (16, 512), (511, 512), (512, 512), (513, 512),
        (8191, 8192), (8192, 8192), (16384, 8192), (100, 100), (250, 100), (5000, 1536), (65535, 65536),
        (70000, 16384), (20000, 7), (1, 1), (1000, 1),
    ]
    pk = np.zeros(len(rows), hdfs.PACKET_DTYPE)
    off = out = 0
    for i, (n, b) in enumerate(rows):
        pk[i] = (off, out, n, b)
        off = (off + n + 31) & ~15  # keep a little gap, 16-aligned
        out += (n + b - 1) // b
    payload = oracle.xorshift64_bytes(off + 32, 1234)
    got = run_dev(hdfs, gpu_ctx, payload, pk)
    assert np.array_equal(got, orc.batch(payload, pk, got.size))


def test_payload_at_end_of_allocation(hdfs, gpu_ctx, orc):
    # Chunks that end exactly at the last byte of the device buffer.
    torch = _torch()
    for n, bpc in [(1000, 512), (4096, 4096), (777, 100), (65536, 512)]:
        payload = oracle.xorshift64_bytes(n, n)
        dev = torch.from_numpy(payload).cuda()
        pk = np.array([(0, 0, n, bpc)], hdfs.PACKET_DTYPE)
        m = (n + bpc - 1) // bpc
        out = torch.zeros(m, dtype=torch.int32, device="cuda")
        gpu_ctx.chunks_dev(pk, dev.data_ptr(), out.data_ptr())
        assert np.array_equal(out.cpu().numpy().view(np.uint32), orc.chunks(payload, bpc))


def test_random_batches(hdfs, gpu_ctx, orc):
    rng = np.random.default_rng(2024)
    for trial in range(6):
        npk = int(rng.integers(1, 200))
        bpcs = rng.choice([512, 1024, 2048, 4096, 8192, 100, 1536, 4000], size=npk)
        lens = rng.integers(0, 70000, size=npk)
        pk = np.zeros(npk, hdfs.PACKET_DTYPE)
        off = out = 0
        for i in range(npk):
            align = 16 if rng.random() < 0.8 else 1
            off = (off + align - 1) // align * align
            pk[i] = (off, out, lens[i], bpcs[i])
            off += int(lens[i]) + int(rng.integers(0, 40))
            out += (int(lens[i]) + int(bpcs[i]) - 1) // int(bpcs[i])
        # output ranges assigned in a random packet order (independent of payload order)
        counts = (pk["len"].astype(np.int64) + pk["bpc"] - 1) // pk["bpc"]
        perm = rng.permutation(npk)
        starts = np.zeros(npk, np.int64)
        starts[perm] = np.concatenate([[0], np.cumsum(counts[perm])[:-1]])
        pk["out_idx"] = starts
        payload = oracle.xorshift64_bytes(off + 16, 500 + trial)
        got = run_dev(hdfs, gpu_ctx, payload, pk)
        assert np.array_equal(got, orc.batch(payload, pk, got.size)), trial


@pytest.mark.parametrize("bpc", [512, 1024, 2048, 4096, 8192])
def test_unaligned_fast_tiles(hdfs, gpu_ctx, orc, bpc):
    """Full chunks of power-of-two bpc take the fast tiles at any alignment
    (unaligned dwordx4 buffer loads): 48 packets at every offset mod 16,
    ragged tails, exec and verify against the oracle."""
    torch = _torch()
    n = 48
    pk = np.zeros(n, hdfs.PACKET_DTYPE)
    off = out = 0
    for i in range(n):
        off += i % 16 + 1  # every phase mod 16
        ln = 65536 - (0 if i % 5 else 300)
        pk[i] = (off, out, ln, bpc)
        off += ln
        out += (ln + bpc - 1) // bpc
    tiles, gen = hdfs.debug_plan(pk)
    assert len(tiles) > 0 and all(int(g["len"]) < bpc for g in gen)  # only short tails go general
    payload = oracle.xorshift64_bytes(off + 64, 4000 + bpc)
    want = orc.batch(payload, pk, out)
    assert np.array_equal(run_dev(hdfs, gpu_ctx, payload, pk), want)
    plan = hdfs.Plan(gpu_ctx, pk)
    dev = torch.from_numpy(payload).cuda()
    exp = torch.from_numpy(want.view(np.int32).copy()).cuda()
    exp[out - 1] ^= 1
    res = torch.zeros(2, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    plan.verify(dev.data_ptr(), exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    assert res.cpu().numpy().view(np.uint32).tolist() == [1, out - 1]
    plan.close()


def test_host_path_pageable_and_pinned(hdfs, gpu_ctx, orc):
    """crc32c_batch_host over 64 MiB slices on two alternating stages: 3
    slices (~137 MiB, so each stage is reused), from pageable memory (pinned
    staging) and from pinned memory (copied in place), then mixed bpc with
    ragged tails, then scattered packets through the gather path (2
    slices)."""
    torch = _torch()
    n = 2200
    pk = oracle.uniform_packets(n)
    payload = oracle.xorshift64_bytes(n * 65536, 42)
    want = orc.batch(payload, pk, n * 128)
    assert np.array_equal(gpu_ctx.batch_host(payload, pk), want)
    pinned = torch.from_numpy(payload).pin_memory()
    got = gpu_ctx.batch_host(pinned.numpy(), pk)
    assert np.array_equal(got, want)
    pkm = oracle.mixed_packets(n)
    pkm["len"][::7] -= 100
    wantm = orc.batch(payload, pkm, oracle.total_checksums(pkm))
    assert np.array_equal(gpu_ctx.batch_host(pinned.numpy(), pkm), wantm)
    # scattered packets (gather path) with out_idx in reverse order
    pk2 = oracle.uniform_packets(n, pkt_len=40000, stride=65536)
    pk2["out_idx"] = pk2["out_idx"][::-1].copy()
    want2 = orc.batch(payload, pk2, oracle.total_checksums(pk2))
    assert np.array_equal(gpu_ctx.batch_host(payload, pk2), want2)


@pytest.mark.parametrize("npk", [1, 5, 16, 17])
def test_host_path_zero_copy(hdfs, gpu_ctx, orc, npk):
    """Small pageable host batches (up to 1 MiB: 1, 5 and 16 packets) are
    copied by the CPU into mapped staging that the kernel reads in place (no
    copy command); 17 packets, and pinned buffers, take the copy path.  A
    buffer starting 0 / 5 / 8 bytes off 16-byte alignment, ragged tails
    (general items and tails under 4 bytes), mixed bpc with a padded bpc
    1000; bit-exact against the oracle."""
    torch = _torch()
    pk = oracle.mixed_packets(npk, 65536, (512, 1000, 1536, 4096))
    pk["len"][1::3] -= 777
    pk["len"][2::5] = 65536 - 510  # a 2-byte tail at bpc 512
    per = (pk["len"].astype(np.int64) + pk["bpc"] - 1) // pk["bpc"]
    pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    n = oracle.total_checksums(pk)
    base = oracle.xorshift64_bytes(npk * 65536 + 64, 600 + npk)
    pinned_all = torch.from_numpy(base).pin_memory().numpy()
    for skew in (0, 5, 8):
        for buf in (base, pinned_all):
            view = buf[skew:skew + npk * 65536]
            want = orc.batch(np.ascontiguousarray(view), pk, n)
            got = gpu_ctx.batch_host(view, pk)
            assert np.array_equal(got, want), (npk, skew, buf is pinned_all)


def test_host_path_pinned_runs(hdfs, gpu_ctx, orc):
    """Scattered packets from pinned memory in long contiguous runs go H2D one
    copy per run (crc32c_batch_host): 4 MiB blocks taken in a shuffled
    order (runs going backwards in memory), one block starting 5 bytes off
    16-byte alignment (general path), ragged and mixed-bpc packets, empty
    packets between runs, a 100-byte gap merged into its run; the same
    batch from pageable memory (CPU gather) must give the same checksums."""
    torch = _torch()
    nblk = 40  # 160 MiB: 3 slices of 64 MiB
    payload = oracle.xorshift64_bytes(nblk * (4 << 20) + 4096, 77)
    pinned = torch.from_numpy(payload).pin_memory()
    rng = np.random.default_rng(5)
    order = rng.permutation(nblk)
    rows, out = [], 0
    for j, b in enumerate(order):
        base = int(b) * (4 << 20) + (5 if j == 3 else 0)
        for p in range(64):
            ln = 65536 - (100 if p == 63 else 0)
            bpc = (512, 1024, 4096)[(j + p) % 3] if j % 4 == 1 else 512
            off = base + p * 65536 + (100 if (j == 7 and p == 10) else 0)
            if j == 7 and p >= 10:
                ln = min(ln, base + 64 * 65536 - off)
            rows.append((off, out, ln, bpc))
            out += (ln + bpc - 1) // bpc
        rows.append((0, out, 0, 512))  # an empty packet between runs
    pk = np.array(rows, hdfs.PACKET_DTYPE)
    want = orc.batch(payload, pk, oracle.total_checksums(pk))
    got = gpu_ctx.batch_host(pinned.numpy(), pk)
    assert np.array_equal(got, want)
    assert np.array_equal(gpu_ctx.batch_host(payload, pk), want)


def test_host_calls_from_threads(hdfs, gpu_ctx, orc):
    """libfuse calls from many worker threads (fuse.c:1771): host batches on
    one shared context, per-packet crc32c_chunks on the default context and
    plan executions on per-thread streams, from 6 threads at once (ctypes
    drops the GIL), every result exact."""
    import threading

    torch = _torch()
    pk = oracle.uniform_packets(80)  # 5 MiB
    pays = [oracle.xorshift64_bytes(80 * 65536, 300 + k) for k in range(6)]
    wants = [orc.batch(p, pk, 80 * 128) for p in pays]
    plan = hdfs.Plan(gpu_ctx, pk)
    devs = [torch.from_numpy(p).cuda() for p in pays]
    torch.cuda.synchronize()
    errors = []

    def work(k):
        try:
            s = torch.cuda.Stream()
            out = torch.zeros(80 * 128, dtype=torch.int32, device="cuda")
            for rep in range(4):
                got = gpu_ctx.batch_host(pays[k], pk)
                assert np.array_equal(got, wants[k]), ("batch_host", k, rep)
                pkt = pays[k][rep * 65536:(rep + 1) * 65536]
                assert np.array_equal(hdfs.chunks(pkt, 512), wants[k][rep * 128:(rep + 1) * 128]), ("chunks", k)
                plan.exec(devs[k].data_ptr(), out.data_ptr(), s.cuda_stream)
                s.synchronize()
                assert np.array_equal(out.cpu().numpy().view(np.uint32), wants[k]), ("plan", k, rep)
        except Exception as e:  # reported on the main thread
            errors.append(repr(e))

    th = [threading.Thread(target=work, args=(k,)) for k in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=100)
    plan.close()
    assert not errors, errors


def test_device_address_plan_over_many_buffers(hdfs, gpu_ctx, orc):
    """CRC32C_DEVICE_ADDRESSES: one plan, one launch over packets living in 12
    separate device buffers (HDFS blocks allocated one by one), with ragged
    blocks, one block starting 5 bytes off alignment (general path) and
    mixed bpc: exact against the oracle per packet, exec and verify; a
    non-NULL payload and the host-resident calls are refused."""
    torch = _torch()
    bufs, rows, want = [], [], []
    out = 0
    for k in range(12):
        n = (4 << 20) - (1000 if k % 3 == 0 else 0)
        data = oracle.xorshift64_bytes(n + 16, 700 + k)
        t = torch.from_numpy(data).cuda()
        bufs.append(t)
        skew = 5 if k == 4 else 0
        bpc = (512, 1024, 4096)[k % 3]
        for o in range(skew, n, 65536):
            ln = min(65536, n - o)
            rows.append((t.data_ptr() + o, out, ln, bpc))
            want.append(orc.chunks(data[o:o + ln], bpc))
            out += (ln + bpc - 1) // bpc
    pk = np.array(rows, hdfs.PACKET_DTYPE)
    want = np.concatenate(want)
    plan = hdfs.Plan(gpu_ctx, pk, hdfs.CRC32C_DEVICE_ADDRESSES)
    assert plan.nchecksums == out
    dev_out = torch.full((out,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    plan.exec(0, dev_out.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    assert np.array_equal(dev_out.cpu().numpy().view(np.uint32), want)
    exp = torch.from_numpy(want.view(np.int32).copy()).cuda()
    res = torch.zeros(2, dtype=torch.int32, device="cuda")
    plan.verify(0, exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    assert res.cpu().numpy().view(np.uint32).tolist() == [0, 0xFFFFFFFF]
    exp[out // 2] ^= 1
    plan.verify(0, exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    assert res.cpu().numpy().view(np.uint32).tolist() == [1, out // 2]
    with pytest.raises(hdfs.Crc32cError):
        plan.exec(bufs[0].data_ptr(), dev_out.data_ptr(), stream.cuda_stream)
    plan.close()
    with pytest.raises(hdfs.Crc32cError):
        gpu_ctx.batch_host(np.zeros(16, np.uint8), oracle.uniform_packets(1, pkt_len=16), hdfs.CRC32C_DEVICE_ADDRESSES)


def test_chunks_default_context(hdfs, orc):
    pkt = oracle.xorshift64_bytes(65536, 99)
    assert np.array_equal(hdfs.chunks(pkt, 512), orc.chunks(pkt, 512))
    assert np.array_equal(hdfs.chunks(pkt[:1000], 512, hdfs.CRC32C_BIG_ENDIAN), orc.chunks(pkt[:1000], 512, True))


def test_multi_single_device(hdfs, orc):
    m = hdfs.Multi([0])
    pk = oracle.uniform_packets(256)
    payload = oracle.xorshift64_bytes(256 * 65536, 7)
    assert np.array_equal(m.batch_host(payload, pk, group_packets=64), orc.batch(payload, pk, 256 * 128))
    m.close()


def test_multi_batch_host_dealt_over_contexts(hdfs, orc):
    """crc32c_multi_batch_host's dealing (round-robin groups of packets, one
    host thread and pipeline per device) on real launches: three contexts on
    the box's one GPU stand in for three devices.  A config-4-shaped file
    (32 x 4 MiB blocks) plus ragged blocks, a short last group, bpc 1536
    packets and an unaligned packet, from pinned and pageable memory, equal
    the oracle; group sizes 64 and 3."""
    torch = _torch()
    m = hdfs.Multi([0, 0, 0])
    try:
        pk = oracle.uniform_packets(32 * 64 + 37)
        rng = np.random.default_rng(4)
        pk["len"][rng.choice(pk.size, 40, replace=False)] = rng.integers(1, 65536, 40).astype(np.uint32)
        pk["bpc"][5::97] = 1536
        pk["payload_off"][1000:] += np.uint64(3)  # every packet from here on off 16-byte alignment
        per = (pk["len"].astype(np.uint64) + pk["bpc"] - 1) // pk["bpc"]
        pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
        payload = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 64, 44)
        want = orc.batch(payload, pk, hdfs.total_checksums(pk))
        pinned = torch.from_numpy(payload).pin_memory()
        for group in (64, 3):
            assert np.array_equal(m.batch_host(payload, pk, group_packets=group), want), group
            assert np.array_equal(m.batch_host(pinned.numpy(), pk, group_packets=group), want), group
    finally:
        m.close()


def test_full_size_c2_against_reference_and_properties(hdfs, gpu_ctx, orc):
    """Config 2 at full size: bit-exact against the oracle, plus the
    size-independent properties (CRC of zero and 0xFF chunks, chunk-shift
    invariance)."""
    pk = oracle.uniform_packets(4096)
    payload = oracle.xorshift64_bytes(4096 * 65536, 0xC2)
    payload[:65536] = 0
    payload[65536:131072] = 0xFF
    got = run_dev(hdfs, gpu_ctx, payload, pk)
    assert np.array_equal(got, orc.batch(payload, pk, got.size))
    assert np.all(got[:128] == 0x30FCEDC0)  # crc32c of 512 zero bytes (known answer)
    assert np.all(got[128:256] == orc.crc32c(np.full(512, 0xFF, np.uint8)))
    # shifting the payload by one chunk shifts the checksum vector by one
    got2 = run_dev(hdfs, gpu_ctx, np.ascontiguousarray(payload[512:]), oracle.uniform_packets(4095))
    assert np.array_equal(got2[:127], got[1:128])


def test_batch_beyond_4GiB(hdfs, gpu_ctx, orc):
    """One plan over 4.6 GiB of HBM (payload offsets past 2^31 and 2^32,
    packets straddling both, some 16-byte-misaligned and ragged, bpc 512 and
    1536): every straddling / first / last packet bit-exact against the
    oracle, and the whole checksum vector equal to three plans over its thirds
    (each below 2 GiB, so no offset wraps in them)."""
    torch = _torch()
    rng = np.random.default_rng(0x4614)
    marks = (1 << 31, 1 << 32)
    rows, off = [], 0
    while off < (1 << 32) + (600 << 20):
        n = 65536
        near = any(abs(off - m) < (1 << 20) for m in marks)
        if near:  # ragged and misaligned around the marks
            n = int(rng.integers(1, 65537))
            off += int(rng.integers(0, 16))
        rows.append((off, n, 1536 if near and rng.integers(0, 3) == 0 else 512))
        off += n
    extent = off
    pk = np.zeros(len(rows), hdfs.PACKET_DTYPE)
    out = 0
    for i, (o, n, b) in enumerate(rows):
        pk[i] = (o, out, n, b)
        out += (n + b - 1) // b
    g = torch.Generator(device="cuda")
    g.manual_seed(4614)
    dev = torch.randint(0, 256, (extent,), dtype=torch.uint8, device="cuda", generator=g)
    stream = torch.cuda.current_stream()

    def exec_plan(pks, base):
        n = hdfs.total_checksums(pks)
        res = torch.zeros(max(n, 1), dtype=torch.int32, device="cuda")
        plan = hdfs.Plan(gpu_ctx, pks, 0)
        plan.exec(dev.data_ptr() + base, res.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        plan.close()
        return res.cpu().numpy().view(np.uint32)[:n]

    got = exec_plan(pk, 0)
    check = {0, len(rows) - 1}
    for m in marks:
        check |= {i for i, (o, n, _) in enumerate(rows) if o < m + (1 << 20) and o + n > m - (1 << 20)}
    for i in sorted(check):
        o, n, b = rows[i]
        want = orc.chunks(dev[o:o + n].cpu().numpy(), b)
        assert np.array_equal(got[pk["out_idx"][i]:pk["out_idx"][i] + want.size], want), (i, o, n, b)
    parts = []
    for part in np.array_split(pk, 3):
        part = part.copy()
        base = int(part["payload_off"][0]) & ~15
        part["payload_off"] -= base
        part["out_idx"] -= part["out_idx"][0]
        assert int((part["payload_off"] + part["len"]).max()) < (1 << 31)
        parts.append(exec_plan(part, base))
    assert np.array_equal(got, np.concatenate(parts))
    del dev
    torch.cuda.empty_cache()


@pytest.mark.parametrize("name", ["c1_one_packet", "c3_one_block_4MiB", "c5_mixed_bpc_96", "ragged_tail_257",
                                  "c2_4096_packets", "c5_mixed_bpc_4096", "c4_file_128MiB", "c2_bpc1536"])
def test_golden_batches_verify_clean(hdfs, gpu_ctx, golden, name):
    """crc32c_plan_verify of every golden batch against its own digest-checked
    checksums: no mismatch; one flipped expected value: exactly that one."""
    torch = _torch()
    spec = [b for b in golden["batches"] if b["name"] == name][0]
    pk = golden_batch_packets(spec)
    payload = oracle.xorshift64_bytes(spec["payload_bytes"], spec["seed"])
    got = run_dev(hdfs, gpu_ctx, payload, pk)
    assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == spec["sha256_le"]
    plan = hdfs.Plan(gpu_ctx, pk)
    dev = torch.from_numpy(payload).cuda()
    exp = torch.from_numpy(got.view(np.int32).copy()).cuda()
    res = torch.zeros(2, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    plan.verify(dev.data_ptr(), exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    assert res.cpu().numpy().view(np.uint32).tolist() == [0, 0xFFFFFFFF]
    k = got.size * 2 // 3
    exp[k] ^= 0x40
    plan.verify(dev.data_ptr(), exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    assert res.cpu().numpy().view(np.uint32).tolist() == [1, k]
    plan.close()


def test_kernel_variant_env_has_no_effect(hdfs, golden, monkeypatch):
    """The product library never switches kernels: with the round-1 A/B
    selector set to a wrong-result diagnostic variant, a fresh context still
    computes the golden config-2 digest and verifies clean."""
    monkeypatch.setenv("HDFS_CRC32C_KVARIANT", "3")
    ctx = hdfs.Context(0)
    try:
        spec = [b for b in golden["batches"] if b["name"] == "c2_4096_packets"][0]
        pk = golden_batch_packets(spec)
        payload = oracle.xorshift64_bytes(spec["payload_bytes"], spec["seed"])
        got = run_dev(hdfs, ctx, payload, pk)
        assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == spec["sha256_le"]
    finally:
        ctx.close()


@pytest.mark.parametrize("variant", [0, 1, 2, 5, 9, 41, 42, 43, 44, 45, 46, 47, 48, 49, 51, 52, 53, 54, 55, 60, 61])
def test_debug_library_variants_exact(hdfs, golden, orc, variant):
    """The A/B kernels of libhdfs_crc32c_debug.so that compute checksums (1 =
    positional nibble tables, 2 = 16 waves per CU, 5 = stamped, 9 = 8
    waves, 41-55 = compact image / quarter-unit shapes) are bit-exact through
    crc32c_debug_plan_exec_variant: golden config-2 / mixed / ragged digests,
    a random ragged batch with general tiles, and CHECKSUM_CRC32."""
    torch = _torch()
    name, exact = hdfs.variant_info(variant)
    assert exact and name
    ctx = hdfs.Context(0)
    stream = torch.cuda.current_stream()

    def run(payload, pk, flags=0):
        dev = torch.from_numpy(payload).cuda()
        n = hdfs.total_checksums(pk)
        out = torch.full((max(n, 1),), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        plan = hdfs.Plan(ctx, pk, flags)
        stamps = torch.zeros(4 * 256 * 16, dtype=torch.int64, device="cuda")
        plan.exec_variant(dev.data_ptr(), out.data_ptr(), variant, stamps.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        plan.close()
        return out.cpu().numpy().view(np.uint32)[:n]

    try:
        for nm in ("c2_4096_packets", "c5_mixed_bpc_96", "ragged_tail_257", "c2_bpc1536"):
            spec = [b for b in golden["batches"] if b["name"] == nm][0]
            got = run(oracle.xorshift64_bytes(spec["payload_bytes"], spec["seed"]), golden_batch_packets(spec))
            assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == spec["sha256_le"], nm
        rng = np.random.default_rng(variant)
        pk = oracle.mixed_packets(24)
        pk["bpc"][::4] = 1000
        pk["len"] = rng.integers(0, 65537, pk.size).astype(np.uint32)
        pk["payload_off"] = np.arange(pk.size, dtype=np.uint64) * np.uint64(65536 + 48) + np.uint64(16)
        per = (pk["len"].astype(np.uint64) + pk["bpc"] - 1) // pk["bpc"]
        pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
        payload = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 64, 99 + variant)
        assert np.array_equal(run(payload, pk), orc.batch(payload, pk, hdfs.total_checksums(pk)))
        T = hdfs.CRC32C_TYPE_CRC32
        assert np.array_equal(run(payload, pk, T), oracle.zlib_batch(payload, pk, hdfs.total_checksums(pk)))
    finally:
        ctx.close()


@pytest.mark.parametrize("variant", [82, 83, 84, 85, 86, 87, 88, 95])
def test_debug_quarter_nopad_variants_exact(hdfs, golden, orc, variant):
    """Round 6's A/Bs of the production quarter-unit build (82) and
    small-batch build (84) against the same with the first unit's / tile's
    loads before the table staging (83, 85): like
    the production small-batch builds they carry no padded- or half-tile
    code, so they are exact on the golden config-3 block, the mixed and
    ragged digests and a ragged batch of power-of-two bpc, and refuse a plan
    with padded tiles (bpc 1000)."""
    torch = _torch()
    ctx = hdfs.Context(0)
    stream = torch.cuda.current_stream()

    def run(payload, pk):
        dev = torch.from_numpy(payload).cuda()
        n = hdfs.total_checksums(pk)
        out = torch.full((max(n, 1),), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        plan = hdfs.Plan(ctx, pk)
        try:
            plan.exec_variant(dev.data_ptr(), out.data_ptr(), variant, 0, stream.cuda_stream)
            stream.synchronize()
        finally:
            plan.close()
        return out.cpu().numpy().view(np.uint32)[:n]

    try:
        for nm in ("c3_one_block_4MiB", "c5_mixed_bpc_96", "ragged_tail_257", "c2_4096_packets"):
            spec = [b for b in golden["batches"] if b["name"] == nm][0]
            got = run(oracle.xorshift64_bytes(spec["payload_bytes"], spec["seed"]), golden_batch_packets(spec))
            assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == spec["sha256_le"], nm
        rng = np.random.default_rng(variant)
        pk = oracle.mixed_packets(24)
        pk["len"] = rng.integers(0, 65537, pk.size).astype(np.uint32)
        pk["payload_off"] = np.arange(pk.size, dtype=np.uint64) * np.uint64(65536 + 48) + np.uint64(16)
        per = (pk["len"].astype(np.uint64) + pk["bpc"] - 1) // pk["bpc"]
        pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
        payload = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 64, 99 + variant)
        assert np.array_equal(run(payload, pk), orc.batch(payload, pk, hdfs.total_checksums(pk)))
        padded = oracle.uniform_packets(8, 65536, 1000)
        with pytest.raises(hdfs.Crc32cError):
            run(oracle.xorshift64_bytes(8 * 65536 + 64, 5), padded)
    finally:
        ctx.close()


@pytest.mark.parametrize("variant", [89, 90, 91, 92, 93, 94])
def test_debug_pow2only_small_variants_exact(hdfs, golden, variant):
    """Round 6's small-batch builds without the general-tile code (89
    quarter units + early loads, 90 quarter units, 91 half units): exact on
    the golden config-3 block, the mixed-bpc batch and config 2 (aligned
    whole chunks only), and refusing a plan of tiles off 16-byte alignment."""
    torch = _torch()
    ctx = hdfs.Context(0)
    stream = torch.cuda.current_stream()

    def run(payload, pk):
        dev = torch.from_numpy(payload).cuda()
        n = hdfs.total_checksums(pk)
        out = torch.full((max(n, 1),), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        plan = hdfs.Plan(ctx, pk)
        try:
            plan.exec_variant(dev.data_ptr(), out.data_ptr(), variant, 0, stream.cuda_stream)
            stream.synchronize()
        finally:
            plan.close()
        return out.cpu().numpy().view(np.uint32)[:n]

    try:
        for nm in ("c3_one_block_4MiB", "c5_mixed_bpc_96", "c2_4096_packets"):
            spec = [b for b in golden["batches"] if b["name"] == nm][0]
            got = run(oracle.xorshift64_bytes(spec["payload_bytes"], spec["seed"]), golden_batch_packets(spec))
            assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == spec["sha256_le"], nm
        skewed = oracle.uniform_packets(8)
        skewed["payload_off"] += np.uint64(5)  # (tiles off 16-byte alignment: the general build's)
        with pytest.raises(hdfs.Crc32cError):
            run(oracle.xorshift64_bytes(8 * 65536 + 64, 6), skewed)
    finally:
        ctx.close()


def test_crc32_type_matches_zlib(hdfs, gpu_ctx):
    """CHECKSUM_CRC32 (CRC32C_TYPE_CRC32): same kernel, zlib-polynomial tables;
    per-chunk results equal zlib.crc32 (the reference returns -ENOSYS here,
    hadooprpc.c:629-631).  Fast tiles, general tiles, mixed bpc, ragged
    tails, unaligned packets, big-endian output, host path."""
    ctx = gpu_ctx
    T = hdfs.CRC32C_TYPE_CRC32
    pk = oracle.uniform_packets(64)
    payload = oracle.xorshift64_bytes(64 * 65536, 77)
    want = oracle.zlib_batch(payload, pk, hdfs.total_checksums(pk))
    assert np.array_equal(run_dev(hdfs, ctx, payload, pk, T), want)
    be = run_dev(hdfs, ctx, payload, pk, T | hdfs.CRC32C_BIG_ENDIAN)
    assert np.array_equal(be, want.byteswap())
    rng = np.random.default_rng(40)
    pk = oracle.mixed_packets(30)
    pk["bpc"][1::5] = 1536
    pk["bpc"][2::5] = 700
    pk["len"] = rng.integers(0, 65537, pk.size).astype(np.uint32)
    pk["payload_off"] = np.arange(pk.size, dtype=np.uint64) * np.uint64(65536 + 40) + np.uint64(3)
    per = (pk["len"].astype(np.uint64) + pk["bpc"] - 1) // pk["bpc"]
    pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    payload = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 64, 81)
    want = oracle.zlib_batch(payload, pk, hdfs.total_checksums(pk))
    assert np.array_equal(run_dev(hdfs, ctx, payload, pk, T), want)
    assert np.array_equal(ctx.batch_host(payload, pk, T), want)


@pytest.mark.parametrize("bpcs", [(512, 1024, 4096), (100, 1000, 1536)])
def test_verify_reports_mismatches(hdfs, gpu_ctx, orc, bpcs):
    """Read-side verification (crc32c_plan_verify / crc32c_verify_host): no
    mismatch on intact data; a corrupted payload byte or expected checksum is
    counted and the lowest bad index reported; wire-order expectations with
    CRC32C_BIG_ENDIAN; power-of-two tiles, general tiles and general-path
    chunks."""
    torch = _torch()
    ctx = gpu_ctx
    rng = np.random.default_rng(60 + bpcs[0])
    pk = oracle.mixed_packets(40, bpcs=bpcs)
    pk["len"] = rng.integers(1, 65537, pk.size).astype(np.uint32)
    pk["len"][:20] = 65536  # whole tiles
    per = (pk["len"].astype(np.uint64) + pk["bpc"] - 1) // pk["bpc"]
    pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    payload = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 64, 5 + bpcs[0])
    n = hdfs.total_checksums(pk)
    stream = torch.cuda.current_stream()
    for flags in (0, hdfs.CRC32C_BIG_ENDIAN):
        want = orc.batch(payload, pk, n, big_endian=bool(flags))
        plan = hdfs.Plan(ctx, pk, flags)
        dev = torch.from_numpy(payload).cuda()
        exp = torch.from_numpy(want.view(np.int32).copy()).cuda()
        res = torch.zeros(2, dtype=torch.int32, device="cuda")

        def verify():
            plan.verify(dev.data_ptr(), exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
            stream.synchronize()
            r = res.cpu().numpy().view(np.uint32)
            return int(r[0]), int(r[1])

        assert verify() == (0, 0xFFFFFFFF)
        # corrupt one payload byte inside packet 25 -> its chunk
        p25 = pk[25]
        off = int(p25["len"]) // 2
        dev[int(p25["payload_off"]) + off] ^= 0x01
        bad_idx = int(p25["out_idx"]) + off // int(p25["bpc"])
        assert verify() == (1, bad_idx)
        dev[int(p25["payload_off"]) + off] ^= 0x01
        # corrupt expected checksums 7 (a whole tile) and bad_idx
        exp[7] ^= 0x100
        exp[bad_idx] ^= 0x1
        assert verify() == (2, 7)
        plan.close()
        # host path
        cnt, first = ctx.verify_host(payload, pk, want, flags)
        assert (cnt, first) == (0, None)
        w2 = want.copy()
        w2[[3, n - 1]] ^= 1
        assert ctx.verify_host(payload, pk, w2, flags) == (2, 3)


@pytest.mark.parametrize("npkts", [1, 3, 75, 138, 263, 388])
def test_small_batches(hdfs, gpu_ctx, orc, npkts):
    """Batches with fewer tiles than waves on the chip (8 KiB tiles, 8 per
    64 KiB packet: from 8 tiles on 8 workgroups to 3104 on 256), each with a
    ragged general-path packet: bit-exact, exec and verify."""
    torch = _torch()
    pk = oracle.uniform_packets(npkts)
    pk["len"][-1] = 65536 - 100  # ragged tail
    payload = oracle.xorshift64_bytes(npkts * 65536 + 64, 900 + npkts)
    n = hdfs.total_checksums(pk)
    want = orc.batch(payload, pk, n)
    got = run_dev(hdfs, gpu_ctx, payload, pk)
    assert np.array_equal(got, want)
    plan = hdfs.Plan(gpu_ctx, pk)
    dev = torch.from_numpy(payload).cuda()
    exp = torch.from_numpy(want.view(np.int32).copy()).cuda()
    res = torch.zeros(2, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    plan.verify(dev.data_ptr(), exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    assert res.cpu().numpy().view(np.uint32).tolist() == [0, 0xFFFFFFFF]
    exp[n // 2] ^= 1
    plan.verify(dev.data_ptr(), exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    assert res.cpu().numpy().view(np.uint32).tolist() == [1, n // 2]
    plan.close()


def test_plan_launches_across_streams(hdfs, gpu_ctx, orc):
    """A plan's verification launches share its device slots, so the library
    keeps them in GPU order when the caller alternates streams
    (crc32c_plan_verify doc): exec and verify interleaved on two streams give
    the oracle's checksums and exact mismatch counts every time.  Exec
    launches are not ordered: eight different payloads through one plan on
    two streams at once each get their own checksums."""
    torch = _torch()
    pk = oracle.uniform_packets(64)
    payload = oracle.xorshift64_bytes(64 * 65536, 71)
    want = orc.batch(payload, pk, 64 * 128)
    plan = hdfs.Plan(gpu_ctx, pk)
    dev = torch.from_numpy(payload).cuda()
    exp = torch.from_numpy(want.view(np.int32).copy()).cuda()
    bad = exp.clone()
    bad[[5, 4000]] ^= 1
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.zeros(64 * 128, dtype=torch.int32, device="cuda") for _ in range(8)]
    results = [torch.zeros(2, dtype=torch.int32, device="cuda") for _ in range(16)]
    for i in range(16):
        s = streams[i % 2].cuda_stream
        plan.verify(dev.data_ptr(), (bad if i % 3 == 0 else exp).data_ptr(), results[i].data_ptr(), s)
        if i % 2 == 0:
            plan.exec(dev.data_ptr(), outs[i // 2].data_ptr(), s)
    torch.cuda.synchronize()
    for i in range(16):
        got = results[i].cpu().numpy().view(np.uint32).tolist()
        assert got == ([2, 5] if i % 3 == 0 else [0, 0xFFFFFFFF]), i
    for o in outs:
        assert np.array_equal(o.cpu().numpy().view(np.uint32), want)
    pays = [oracle.xorshift64_bytes(64 * 65536, 200 + k) for k in range(8)]
    devs = [torch.from_numpy(x).cuda() for x in pays]
    torch.cuda.synchronize()
    for k in range(8):
        plan.exec(devs[k].data_ptr(), outs[k].data_ptr(), streams[k % 2].cuda_stream)
    torch.cuda.synchronize()
    for k in range(8):
        assert np.array_equal(outs[k].cpu().numpy().view(np.uint32), orc.batch(pays[k], pk, 64 * 128)), k
    plan.close()


@pytest.mark.parametrize("flags", [0, 0x20])  # (0x20: CRC32C_COUNT_COMPLETION, the counters gate reuse)
def test_plans_destroyed_in_flight_and_recycled(hdfs, orc, flags):
    """Plan descriptors come from a recycled pool and are uploaded
    asynchronously: 100 plans of different shapes are each created, launched
    at once on a fresh non-blocking stream (the launch must wait for the
    upload) and destroyed while their launch may still run; their blocks are
    reused by later plans only after an epoch.  Every output is exact."""
    torch = _torch()
    ctx = hdfs.Context(0)
    rng = np.random.default_rng(5)
    s = torch.cuda.Stream()
    jobs = []
    try:
        for i in range(100):
            npk = int(rng.integers(1, 40))
            pk = oracle.uniform_packets(npk, pkt_len=int(rng.integers(1, 65537)), bpc=int(rng.choice([512, 1536, 4096])),
                                        stride=65536 + 16)
            n = hdfs.total_checksums(pk)
            payload = oracle.xorshift64_bytes(npk * (65536 + 16) + 64, 900 + i)
            dev = torch.from_numpy(payload).cuda()
            out = torch.full((max(n, 1),), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            plan = hdfs.Plan(ctx, pk, flags)
            plan.exec(dev.data_ptr(), out.data_ptr(), s.cuda_stream)
            plan.close()  # (launch possibly still in flight)
            jobs.append((payload, pk, n, dev, out))
        torch.cuda.synchronize()
        for payload, pk, n, _, out in jobs:
            assert np.array_equal(out.cpu().numpy().view(np.uint32)[:n], orc.batch(payload, pk, n))
    finally:
        ctx.close()


def test_plan_destroyed_after_its_stream(hdfs, orc):
    """with CRC32C_COUNT_COMPLETION a C caller (a FUSE
    daemon with per-thread streams) may destroy a launch stream BEFORE the
    plan launched on it -- plan destroy touches no stream; the plan's block
    returns to the pool once its launches' workgroups have counted
    themselves complete (the completion counters).  Raw HIP streams (torch pools its streams and never destroys
    them): each plan is launched on a fresh stream, the stream destroyed at
    once (its launch may still run), then the plan destroyed; later plans
    reuse the destroyed plans' blocks, and every output is exact."""
    import ctypes

    torch = _torch()
    hip = ctypes.CDLL("libamdhip64.so")  # (the process's HIP runtime, loaded by torch)
    ctx = hdfs.Context(0)
    pk = oracle.uniform_packets(8)
    n = hdfs.total_checksums(pk)
    try:
        blocks, seen_again, jobs = set(), 0, []
        for i in range(60):
            payload = oracle.xorshift64_bytes(8 * 65536, 4400 + i)
            dev = torch.from_numpy(payload).cuda()
            out = torch.full((n,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            plan = hdfs.Plan(ctx, pk, hdfs.CRC32C_COUNT_COMPLETION)
            blk = int(hdfs.lib().crc32c_debug_plan_block(plan.handle))
            seen_again += blk in blocks
            blocks.add(blk)
            s = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(s)) == 0
            plan.exec(dev.data_ptr(), out.data_ptr(), s.value)
            assert hip.hipStreamDestroy(s) == 0  # (before the plan; its launch may still run)
            plan.close()
            jobs.append((payload, dev, out))
            if i % 10 == 9:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        for payload, _, out in jobs:
            assert np.array_equal(out.cpu().numpy().view(np.uint32), orc.batch(payload, pk, n))
        assert seen_again > 0, "no destroyed plan's block was reused"
    finally:
        ctx.close()


def test_plan_destroyed_after_its_context(hdfs, orc):
    """A plan outliving crc32c_ctx_destroy (a garbage collector freeing a
    plan late, e.g. one a failed test's traceback held): the context is
    reference-counted by its plans, so the late destroy returns the plan's
    block to a still-live pool; the context's teardown is deferred past its
    last plan (a plan destroy never synchronises) to the next context
    create that finds its work done, or the next context destroy."""
    torch = _torch()
    pk = oracle.uniform_packets(8)
    n = hdfs.total_checksums(pk)
    payload = oracle.xorshift64_bytes(8 * 65536, 31337)
    dev = torch.from_numpy(payload).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    for _ in range(3):
        ctx = hdfs.Context(0)
        plans = [hdfs.Plan(ctx, pk) for _ in range(3)]
        for p in plans:
            p.exec(dev.data_ptr(), out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        ctx.close()  # (the plans still hold it)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), orc.batch(payload, pk, n))
        plans[0].exec(dev.data_ptr(), out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        for p in plans:
            p.close()
        torch.cuda.synchronize()


@pytest.mark.parametrize("bpc", [512, 2048, 4096])
def test_shifted_tiles_large_batch(hdfs, gpu_ctx, orc, bpc):
    """A batch large enough for the full-image general build (> 16 tiles per
    CU), every packet at a different offset mod 16 with partial last tiles:
    the tiles off 16-byte alignment load from the aligned address below and
    reassemble each lane's bytes (wave shift + alignbyte, the tile's last 16
    bytes loaded apart).  Exec and verify against the oracle."""
    torch = _torch()
    n = 720
    pk = np.zeros(n, hdfs.PACKET_DTYPE)
    off = out = 0
    for i in range(n):
        off += i % 16 + 1  # every phase mod 16
        ln = 65536 - (i % 7) * 512 * (bpc // 512) - (i % 3) * 37
        pk[i] = (off, out, ln, bpc)
        off += ln
        out += (ln + bpc - 1) // bpc
    tiles, _ = hdfs.debug_plan(pk)
    assert len(tiles) > 16 * 256 and np.any(tiles["src"] & np.uint64(15))
    payload = oracle.xorshift64_bytes(off + 64, 7000 + bpc)
    want = orc.batch(payload, pk, out)
    assert np.array_equal(run_dev(hdfs, gpu_ctx, payload, pk), want)
    plan = hdfs.Plan(gpu_ctx, pk)
    dev = torch.from_numpy(payload).cuda()
    exp = torch.from_numpy(want.view(np.int32).copy()).cuda()
    exp[[7, out - 1]] ^= 1
    res = torch.zeros(2, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    plan.verify(dev.data_ptr(), exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    assert res.cpu().numpy().view(np.uint32).tolist() == [2, 7]
    plan.close()


@pytest.mark.parametrize("seed", [11, 12, 13, 14])
def test_fuzz_mixed_batches(hdfs, gpu_ctx, orc, seed):
    """Seeded random batches that mix every work-item kind the plan can
    build -- power-of-two tiles at any alignment (shifted or not), general
    items (padded and unpadded bpc, tails riding behind full chunks, chunks
    spanning subtiles), padded power-of-two tiles, half tiles, GenItems
    (tails under 4 bytes, bpc > 8192) -- at sizes that select each kernel
    build (quarter units, compact image, full image; half-tile builds with
    and without shifted loads); exec and verify against the oracle."""
    torch = _torch()
    rng = np.random.default_rng(seed)
    for size in (12, 90, 700):  # packets: quarter-unit, compact and full-image builds
        bpcs = rng.choice([512, 1024, 4096, 8192, 1536, 1000, 100, 3000, 513, 9000, 700, 1100, 2000, 256],
                          size=size)
        pk = np.zeros(size, hdfs.PACKET_DTYPE)
        off = out = 0
        for i in range(size):
            bpc = int(bpcs[i])
            off += int(rng.integers(16, 48)) if rng.random() < 0.5 else 16 - off % 16 + 16
            ln = int(rng.integers(1, 65537)) if rng.random() < 0.4 else 65536 - int(rng.integers(0, 4)) * bpc
            ln = max(ln, 1)
            pk[i] = (off, out, ln, bpc)
            off += ln
            out += (ln + bpc - 1) // bpc
        payload = oracle.xorshift64_bytes(off + 64, 100 * seed + size)
        want = orc.batch(payload, pk, out)
        got = run_dev(hdfs, gpu_ctx, payload, pk)
        assert np.array_equal(got, want), (size, np.nonzero(got != want)[0][:8])
        plan = hdfs.Plan(gpu_ctx, pk)
        dev = torch.from_numpy(payload).cuda()
        exp = torch.from_numpy(want.view(np.int32).copy()).cuda()
        bad = int(rng.integers(0, out))
        exp[bad] ^= 0x40
        res = torch.zeros(2, dtype=torch.int32, device="cuda")
        stream = torch.cuda.current_stream()
        plan.verify(dev.data_ptr(), exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        assert res.cpu().numpy().view(np.uint32).tolist() == [1, bad], size
        plan.close()


@pytest.mark.parametrize("npk", [64, 96, 112, 128, 192, 224, 256])
def test_small_batch_builds_by_size(hdfs, gpu_ctx, orc, npk):
    """Batches of bpc 512 / 1024 / 4096 packets (ragged tails, skewed
    offsets) sized to select each small-batch build: quarter units with the
    first unit's loads before the staging (64 packets: 512 tiles, <= 2 per
    CU), quarter units (96), half units (112-192: 3-6 tiles per CU), whole
    tiles on the compact image (224, 256); exec and verify (one flipped
    checksum) against the oracle."""
    torch = _torch()
    rng = np.random.default_rng(npk)
    pk = oracle.mixed_packets(npk)
    pk["len"][3::7] = rng.integers(1, 65536, pk["len"][3::7].size).astype(np.uint32)
    pk["payload_off"] = np.arange(npk, dtype=np.uint64) * np.uint64(65536 + 64) + np.uint64(5) * (
        np.arange(npk, dtype=np.uint64) % np.uint64(3))
    per = (pk["len"].astype(np.uint64) + pk["bpc"] - 1) // pk["bpc"]
    pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    n = int(per.sum())
    payload = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 64, 700 + npk)
    want = orc.batch(payload, pk, n)
    got = run_dev(hdfs, gpu_ctx, payload, pk)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]
    plan = hdfs.Plan(gpu_ctx, pk)
    dev = torch.from_numpy(payload).cuda()
    exp = torch.from_numpy(want.view(np.int32).copy()).cuda()
    bad = int(rng.integers(0, n))
    exp[bad] ^= 0x100
    res = torch.zeros(2, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    plan.verify(dev.data_ptr(), exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    assert res.cpu().numpy().view(np.uint32).tolist() == [1, bad]
    plan.close()


def test_entry_points_reject_bad_arguments(hdfs, gpu_ctx):
    """The C ABI's argument checks on the GPU path: -EINVAL (never a launch)
    for NULL plans / results / expected arrays, unknown flags, bpc 0, a
    checksum range past 2^32, a buffer-list range past its buffers, and a
    device-address plan given a payload pointer."""
    import ctypes
    import errno

    torch = _torch()
    L = hdfs.lib()
    vp = ctypes.c_void_p
    pk = oracle.uniform_packets(2)
    plan = hdfs.Plan(gpu_ctx, pk)
    dev = torch.zeros(2 * 65536, dtype=torch.uint8, device="cuda")
    res = torch.zeros(2, dtype=torch.int32, device="cuda")
    exp = torch.zeros(256, dtype=torch.int32, device="cuda")
    bits = torch.zeros(8, dtype=torch.int32, device="cuda")
    inval = -errno.EINVAL
    assert L.crc32c_plan_verify_bitmap(None, vp(dev.data_ptr()), vp(exp.data_ptr()), vp(res.data_ptr()),
                                       vp(bits.data_ptr()), None) == inval
    assert L.crc32c_plan_verify_bitmap(plan.handle, vp(dev.data_ptr()), vp(exp.data_ptr()), None,
                                       vp(bits.data_ptr()), None) == inval
    assert L.crc32c_plan_verify_bitmap(plan.handle, vp(dev.data_ptr()), None, vp(res.data_ptr()),
                                       vp(bits.data_ptr()), None) == inval
    assert L.crc32c_plan_exec(None, vp(dev.data_ptr()), vp(exp.data_ptr()), None) == inval
    plan.close()
    bad = pk.copy()
    bad["bpc"][1] = 0
    with pytest.raises(hdfs.Crc32cError) as e:
        hdfs.Plan(gpu_ctx, bad)
    assert e.value.rc == inval
    bad = pk.copy()
    bad["out_idx"][1] = (1 << 32) - 10
    with pytest.raises(hdfs.Crc32cError):
        hdfs.Plan(gpu_ctx, bad)
    with pytest.raises(hdfs.Crc32cError) as e:
        hdfs.Plan(gpu_ctx, pk, 1 << 30)  # unknown flag
    assert e.value.rc == inval
    with pytest.raises(hdfs.Crc32cError) as e:
        gpu_ctx.write_plan([(dev.data_ptr(), 1000)], 10, 1000)  # past the buffers
    assert e.value.rc == inval
    aplan = hdfs.Plan(gpu_ctx, np.array([(dev.data_ptr(), 0, 512, 512)], hdfs.PACKET_DTYPE),
                      hdfs.CRC32C_DEVICE_ADDRESSES)
    with pytest.raises(hdfs.Crc32cError):
        aplan.exec(dev.data_ptr(), exp.data_ptr(), 0)  # a device-address plan takes payload NULL
    aplan.exec(0, exp.data_ptr(), 0)
    torch.cuda.synchronize()
    aplan.close()


PADDED_BPCS = [4, 100, 511, 513, 700, 1000, 1023, 1537, 2000, 2047, 3585, 4000, 4095, 7681, 8000, 8191]


@pytest.mark.parametrize("npk", [3, 40, 600])
def test_padded_power_of_two_tiles(hdfs, gpu_ctx, orc, npk):
    """Chunks of bpc = 512 * 2^lg - pad run as padded power-of-two tiles
    (round 5): every pad class of lg = 0..4, packets with and without a tail
    chunk, first chunks at offsets < 16 (those take a GenItem) and at odd
    offsets; 3 / 40 packets run the compact builds, 600 the full image; exec
    in both byte orders and verify (clean, a corrupted payload byte, a
    corrupted expectation) bit-exact against the reference."""
    torch = _torch()
    rng = np.random.default_rng(1700 + npk)
    pk = np.zeros(npk, oracle.PACKET_DTYPE)
    pk["bpc"] = rng.choice(PADDED_BPCS, npk)
    pk["len"] = np.where(rng.random(npk) < 0.5, 65536, rng.integers(1, 65537, npk))
    gaps = rng.integers(0, 41, npk)
    gaps[0] = rng.integers(0, 21)
    pk["payload_off"] = np.cumsum(gaps) + np.concatenate([[0], np.cumsum(pk["len"].astype(np.int64))[:-1]])
    per = (pk["len"].astype(np.uint64) + pk["bpc"] - 1) // pk["bpc"]
    pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    tiles, _ = hdfs.debug_plan(pk)
    meta = tiles["meta"].astype(np.int64)
    assert np.any(((meta >> 18) & 511) & ~(meta >> 31))  # some padded power-of-two tiles
    payload = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 64, 1800 + npk)
    n = hdfs.total_checksums(pk)
    for flags in (0, hdfs.CRC32C_BIG_ENDIAN):
        want = orc.batch(payload, pk, n, big_endian=bool(flags))
        assert np.array_equal(run_dev(hdfs, gpu_ctx, payload, pk, flags), want)
        assert np.array_equal(run_dev(hdfs, gpu_ctx, payload, pk, flags, offset=5), want)
    want = orc.batch(payload, pk, n)
    plan = hdfs.Plan(gpu_ctx, pk)
    dev = torch.from_numpy(payload).cuda()
    exp = torch.from_numpy(want.view(np.int32).copy()).cuda()
    res = torch.zeros(2, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def verify():
        plan.verify(dev.data_ptr(), exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        return res.cpu().numpy().view(np.uint32).tolist()

    assert verify() == [0, 0xFFFFFFFF]
    p = pk[npk // 2]
    off = int(p["len"]) // 3
    dev[int(p["payload_off"]) + off] ^= 0x40
    bad = int(p["out_idx"]) + off // int(p["bpc"])
    assert verify() == [1, bad]
    dev[int(p["payload_off"]) + off] ^= 0x40
    exp[n - 1] ^= 1
    assert verify() == [1, n - 1]
    plan.close()


@pytest.mark.parametrize("bpc", [1000, 4000, 300])
def test_padded_tiles_multi_block_launch(hdfs, gpu_ctx, orc, bpc):
    """crc32c_plan_exec_blocks with a one-block plan of padded tiles over
    blocks at 16-byte-aligned and odd device addresses."""
    torch = _torch()
    pk = oracle.uniform_packets(64)
    pk["bpc"] = bpc
    per = (pk["len"].astype(np.uint64) + bpc - 1) // bpc
    pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    n = hdfs.total_checksums(pk)
    block = 64 * 65536
    offs = [0, block + 64, 2 * block + 205]
    dev = torch.zeros(3 * block + 512, dtype=torch.uint8, device="cuda")
    wants = []
    for b, o in enumerate(offs):
        host = oracle.xorshift64_bytes(block, 2000 + b)
        dev[o:o + block].copy_(torch.from_numpy(host))
        wants.append(orc.batch(host, pk, n))
    outs = torch.zeros((3, n), dtype=torch.int32, device="cuda")
    plan = hdfs.Plan(gpu_ctx, pk)
    stream = torch.cuda.current_stream()
    plan.exec_blocks([dev.data_ptr() + o for o in offs], [outs[b].data_ptr() for b in range(3)], stream.cuda_stream)
    stream.synchronize()
    plan.close()
    got = outs.cpu().numpy().view(np.uint32)
    for b in range(3):
        assert np.array_equal(got[b], wants[b]), b


HALF_BPCS = [4, 17, 100, 200, 255, 256, 513, 600, 700, 767, 768, 1025, 1100, 1280]


@pytest.mark.parametrize("npk", [3, 40, 600])
def test_half_tiles(hdfs, gpu_ctx, orc, npk):
    """bpc <= 256 and 512 < bpc <= 768 run as half tiles (round 5: two
    chunks' partial parts per 512-byte block, the lower half on the columns
    q + 16): packets with and without a tail chunk, first chunks at offsets
    < 16 and odd offsets, both byte orders, verify with a corrupted payload
    byte and a corrupted expectation; bit-exact against the reference."""
    torch = _torch()
    rng = np.random.default_rng(1900 + npk)
    pk = np.zeros(npk, oracle.PACKET_DTYPE)
    pk["bpc"] = rng.choice(HALF_BPCS, npk)
    pk["len"] = np.where(rng.random(npk) < 0.5, 65536, rng.integers(1, 65537, npk))
    gaps = rng.integers(0, 41, npk)
    gaps[0] = rng.integers(0, 21)
    pk["payload_off"] = np.cumsum(gaps) + np.concatenate([[0], np.cumsum(pk["len"].astype(np.int64))[:-1]])
    per = (pk["len"].astype(np.uint64) + pk["bpc"] - 1) // pk["bpc"]
    pk["out_idx"] = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint64)
    tiles, _ = hdfs.debug_plan(pk)
    meta = tiles["meta"].astype(np.int64)
    assert np.any((meta >> 30) == 1)  # some half tiles
    payload = oracle.xorshift64_bytes(int((pk["payload_off"] + pk["len"]).max()) + 64, 2100 + npk)
    n = hdfs.total_checksums(pk)
    for flags in (0, hdfs.CRC32C_BIG_ENDIAN):
        want = orc.batch(payload, pk, n, big_endian=bool(flags))
        assert np.array_equal(run_dev(hdfs, gpu_ctx, payload, pk, flags), want)
        assert np.array_equal(run_dev(hdfs, gpu_ctx, payload, pk, flags, offset=7), want)
    want = orc.batch(payload, pk, n)
    plan = hdfs.Plan(gpu_ctx, pk)
    dev = torch.from_numpy(payload).cuda()
    exp = torch.from_numpy(want.view(np.int32).copy()).cuda()
    res = torch.zeros(2, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def verify():
        plan.verify(dev.data_ptr(), exp.data_ptr(), res.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        return res.cpu().numpy().view(np.uint32).tolist()

    assert verify() == [0, 0xFFFFFFFF]
    p = pk[npk // 2]
    off = int(p["len"]) // 3
    dev[int(p["payload_off"]) + off] ^= 0x02
    bad = int(p["out_idx"]) + off // int(p["bpc"])
    assert verify() == [1, bad]
    dev[int(p["payload_off"]) + off] ^= 0x02
    exp[0] ^= 1
    assert verify() == [1, 0]
    plan.close()


@pytest.mark.parametrize("bpc", [700, 100, 768, 256, 1100])
def test_half_tiles_multi_block_launch(hdfs, gpu_ctx, orc, bpc):
    """crc32c_plan_exec_blocks with a one-block plan of half tiles over blocks
    at 16-byte-aligned and odd device addresses."""
    test_padded_tiles_multi_block_launch(hdfs, gpu_ctx, orc, bpc)
