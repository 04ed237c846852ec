#!/usr/bin/env python3
"""Soak run of the production path: random batches mixing every work-item
kind (the GPU fuzz test's generator, plus CRC32 and wire-order flags and a
batch size that selects each kernel build) and random FUSE-shaped
buffer-list write plans (NULL zero fill, chunks spanning buffers), each
executed on one of two streams and verified with a mismatch bitmap against
k random flipped checksums, every result checked against the oracle.
Writes a progress line every ~10 s (and the summary at the end) to --out.

    python tools/soak.py [--seconds 300] [--out gpurun_out/soak.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def batch(hdfs, rng, size):
    bpcs = rng.choice([512, 1024, 2048, 4096, 8192, 1536, 1000, 100, 3000, 513, 9000, 700, 2000, 4000, 256, 768, 7681],
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
    return pk, off + 64, out


def write_sums(orc, stream, bo, length, blockoffset, psize, bpc):
    """hadoop_rpc_send_packets' checksums over the assembled stream (oracle)."""
    out, pos, sent = [], bo, 0
    while True:
        plen = min(length - sent, psize)
        past = (blockoffset + sent) % bpc
        if plen > 0 and past:
            plen = min(bpc - past, length - sent)
        if plen == 0:
            break
        out.append(orc.chunks(stream[pos:pos + plen], bpc))
        pos += plen
        sent += plen
    return np.concatenate(out) if out else np.zeros(0, np.uint32)


def write_round(torch, hdfs, orc, ctx, rng, stream):
    """One random buffer-list write plan (1-6 buffers, NULL or data, any skew)
    exec'd and verified with a bitmap; True when exact."""
    import oracle

    nb = int(rng.integers(1, 7))
    bufs, parts, keep = [], [], []
    for _ in range(nb):
        n = int(rng.integers(0, 400000))
        if rng.random() < 0.3:
            bufs.append((0, n))
            parts.append(np.zeros(n, np.uint8))
        else:
            d = oracle.xorshift64_bytes(n + 32, int(rng.integers(1 << 62)))
            skew = int(rng.integers(0, 16))
            t = torch.from_numpy(d).cuda()
            keep.append(t)
            bufs.append((t.data_ptr() + skew, n))
            parts.append(d[skew:skew + n])
    sb = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    bo = int(rng.integers(0, sb.size // 3 + 1))
    length = int(rng.integers(0, sb.size - bo + 1))
    bpc = int(rng.choice([512, 1024, 4096, 100, 1536, 700, 1000]))
    blockoffset = int(rng.integers(0, 3)) * int(rng.integers(0, 1 << 20))
    psize = int(rng.choice([65536, bpc * 7]))
    want = write_sums(orc, sb, bo, length, blockoffset, psize, bpc)
    plan = ctx.write_plan(bufs, bo, length, blockoffset, psize, bpc)
    n = want.size
    ok = plan.nchecksums == n
    if ok and n:
        out = torch.full((n,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        stream.wait_stream(torch.cuda.current_stream())  # (the buffers' copies, out's fill)
        plan.exec(0, out.data_ptr(), stream.cuda_stream)
        flips = sorted(set(int(x) for x in rng.integers(0, n, int(rng.integers(0, 4)))))
        exp = want.copy()
        for i in flips:
            exp[i] ^= np.uint32(0x100)
        d_exp = torch.from_numpy(exp.view(np.int32)).cuda()
        res = torch.zeros(2, dtype=torch.int32, device="cuda")
        bits = torch.full(((n + 31) // 32,), -1, dtype=torch.int32, device="cuda")
        stream.wait_stream(torch.cuda.current_stream())
        plan.verify(0, d_exp.data_ptr(), res.data_ptr(), stream.cuda_stream, dev_bad_bits=bits.data_ptr())
        torch.cuda.synchronize()
        b = np.unpackbits(bits.cpu().numpy().view(np.uint8), bitorder="little")
        ok = (np.array_equal(out.cpu().numpy().view(np.uint32), want)
              and res.cpu().numpy().view(np.uint32).tolist() == [len(flips), flips[0] if flips else 0xFFFFFFFF]
              and np.flatnonzero(b).tolist() == flips)
    plan.close()
    return ok, n, length


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=300)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "soak.jsonl"))
    ap.add_argument("--seed", type=int, default=7)
    args = ap.parse_args()
    import torch

    import oracle
    from bench import load_package

    hdfs = load_package()
    hdfs.lib()
    orc = oracle.Oracle()
    ctx = hdfs.Context(0)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    rng = np.random.default_rng(args.seed)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    log = open(args.out, "w")
    stats = {"batches": 0, "checksums": 0, "bytes": 0, "mismatching_results": 0, "verify_bits_checked": 0}
    t0 = last = time.time()
    stats["write_plans"] = 0
    while time.time() - t0 < args.seconds:
        if rng.random() < 0.3:  # a FUSE-shaped buffer-list write plan
            ok, n, nbytes = write_round(torch, hdfs, orc, ctx, rng, streams[int(rng.integers(0, 2))])
            stats["write_plans"] += 1
            stats["checksums"] += n
            stats["bytes"] += nbytes
            stats["verify_bits_checked"] += n
            if not ok:
                stats["mismatching_results"] += 1
                log.write(json.dumps({"FAIL": True, "write_plan": True}) + "\n")
                log.flush()
            continue
        size = int(rng.choice([3, 12, 90, 700, 3000]))
        pk, extent, n = batch(hdfs, rng, size)
        flags = 0
        if rng.random() < 0.3:
            flags |= hdfs.CRC32C_TYPE_CRC32
        if rng.random() < 0.3:
            flags |= hdfs.CRC32C_BIG_ENDIAN
        payload = oracle.xorshift64_bytes(extent, int(rng.integers(1 << 62)))
        if flags & hdfs.CRC32C_TYPE_CRC32:
            want = oracle.zlib_batch(payload, pk, n)
            if flags & hdfs.CRC32C_BIG_ENDIAN:
                want = want.byteswap()
        else:
            want = orc.batch(payload, pk, n, big_endian=bool(flags & hdfs.CRC32C_BIG_ENDIAN))
        s = streams[int(rng.integers(0, 2))]
        dev = torch.from_numpy(payload).cuda()
        out = torch.full((max(n, 1),), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        plan = hdfs.Plan(ctx, pk, flags)
        s.wait_stream(torch.cuda.current_stream())  # (the payload's copy, out's fill)
        plan.exec(dev.data_ptr(), out.data_ptr(), s.cuda_stream)
        flips = sorted(set(int(x) for x in rng.integers(0, n, int(rng.integers(0, 6)))))
        exp = want.copy()
        for i in flips:
            exp[i] ^= np.uint32(1 << int(rng.integers(0, 32)))
        d_exp = torch.from_numpy(exp.view(np.int32)).cuda()
        res = torch.zeros(2, dtype=torch.int32, device="cuda")
        bits = torch.full(((n + 31) // 32,), -1, dtype=torch.int32, device="cuda")
        s2 = streams[int(rng.integers(0, 2))]
        s2.wait_stream(torch.cuda.current_stream())  # (the expected values' copy)
        plan.verify(dev.data_ptr(), d_exp.data_ptr(), res.data_ptr(), s2.cuda_stream, dev_bad_bits=bits.data_ptr())
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)[:n]
        r = res.cpu().numpy().view(np.uint32).tolist()
        b = np.unpackbits(bits.cpu().numpy().view(np.uint8), bitorder="little")
        ok = (np.array_equal(got, want) and r == [len(flips), flips[0] if flips else 0xFFFFFFFF]
              and np.flatnonzero(b).tolist() == flips)
        plan.close()
        stats["batches"] += 1
        stats["checksums"] += n
        stats["bytes"] += int(pk["len"].astype(np.int64).sum())
        stats["verify_bits_checked"] += n
        if not ok:
            stats["mismatching_results"] += 1
            log.write(json.dumps({"FAIL": True, "size": size, "flags": flags, "flips": flips, "verify": r,
                                  "bad_exec": np.flatnonzero(got != want)[:8].tolist()}) + "\n")
            log.flush()
        if time.time() - last > 10:
            last = time.time()
            log.write(json.dumps(dict(stats, elapsed_s=round(last - t0, 1))) + "\n")
            log.flush()
    summary = dict(stats, elapsed_s=round(time.time() - t0, 1), done=True)
    log.write(json.dumps(summary) + "\n")
    log.close()
    ctx.close()
    print(json.dumps(summary))
    return 1 if stats["mismatching_results"] else 0


if __name__ == "__main__":
    sys.exit(main())
