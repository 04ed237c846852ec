#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE itself.

The expected values come from ``/root/reference/src/crc32c.c`` compiled where
it lies (``oracle/Makefile`` -> ``oracle/_ref/``), called exactly as the packet
writer calls it (``src/hadooprpc.c:733-742``), and from the reference's own
``#ifdef TEST`` stdin harness (``src/crc32c.c:345-382``).  Fixtures hold only
seeds, shapes and expected outputs -- payloads are regenerated from the
documented xorshift64 stream (``oracle.xorshift64_bytes``).

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def hx(v: int) -> str:
    return "%08x" % v


def fill(kind: str, n: int, seed: int) -> np.ndarray:
    if kind == "xorshift":
        return oracle.xorshift64_bytes(n, seed)
    if kind == "zero":
        return np.zeros(n, np.uint8)
    if kind == "ff":
        return np.full(n, 0xFF, np.uint8)
    if kind == "ramp":
        return (np.arange(n) & 0xFF).astype(np.uint8)
    raise ValueError(kind)


def main() -> None:
    oracle.build()
    ref = oracle.Reference()

    # 1. Known answers: published vectors (RFC 3720 B.4, the "check" value of
    #    CRC-32C) plus zero/ramp strings; each is ALSO re-derived here from the
    #    reference so a transcription error cannot hide.
    published = [
        {"name": "check_123456789", "hex": b"123456789".hex(), "crc": "e3069283", "source": "CRC-32C check value"},
        {"name": "rfc3720_zeros32", "hex": "00" * 32, "crc": "8a9136aa", "source": "RFC 3720 B.4"},
        {"name": "rfc3720_ones32", "hex": "ff" * 32, "crc": "62a8ab43", "source": "RFC 3720 B.4"},
        {"name": "rfc3720_incr32", "hex": bytes(range(32)).hex(), "crc": "46dd794e", "source": "RFC 3720 B.4"},
        {"name": "rfc3720_decr32", "hex": bytes(range(31, -1, -1)).hex(), "crc": "113fdb5c", "source": "RFC 3720 B.4"},
    ]
    for e in published:
        got = hx(ref.crc32c(bytes.fromhex(e["hex"])))
        assert got == e["crc"], (e["name"], got)
    derived = []
    for n in [0, 1, 3, 4, 7, 8, 9, 15, 16, 17, 255, 256, 511, 512, 513, 767, 768, 1024, 4096, 65536]:
        derived.append({"name": "zeros_%d" % n, "kind": "zero", "len": n, "crc": hx(ref.crc32c(bytes(n)))})
    for n in [512, 4096]:
        derived.append({"name": "ramp_%d" % n, "kind": "ramp", "len": n, "crc": hx(ref.crc32c(fill("ramp", n, 0)))})
    derived.append({"name": "ones_512", "kind": "ff", "len": 512, "crc": hx(ref.crc32c(b"\xff" * 512))})
    # incremental crc argument (crc32c.c:237: the argument is a finished CRC)
    chained = []
    for n, split in [(512, 256), (1000, 3), (4096, 1537), (70000, 65536)]:
        buf = fill("xorshift", n, oracle.SEED + n)
        c1 = ref.crc32c(buf[:split])
        chained.append(
            {"seed": oracle.SEED + n, "len": n, "split": split, "first": hx(c1), "crc": hx(ref.crc32c(buf[split:], c1)),
             "oneshot": hx(ref.crc32c(buf))}
        )
        assert chained[-1]["crc"] == chained[-1]["oneshot"]

    # The reference's own stdin harness: 786432-byte slices chained through
    # the crc argument (crc32c.c:347-373), hardware and software paths.
    harness = []
    test_bin = os.path.join(oracle.HERE, "_ref", "crc32c_test")
    for n, seed in [(3 * 786432 + 12345, 7), (1 << 20, 11)]:
        data = fill("xorshift", n, seed).tobytes()
        hw = subprocess.run([test_bin], input=data, capture_output=True, check=True).stdout.decode().strip()
        sw = subprocess.run([test_bin, "sw"], input=data, capture_output=True, check=True).stdout.decode().strip()
        assert hw == sw
        harness.append({"seed": seed, "len": n, "crc": hw})

    with open(os.path.join(OUT, "known_answers.json"), "w") as f:
        json.dump({"published": published, "derived": derived, "chained": chained, "stdin_harness": harness}, f, indent=1)

    # 2. Seeded single packets through the chunk loop (hadooprpc.c:733-742),
    #    per bpc, with the edge cases the write path produces: short tail,
    #    len < bpc (first packet trimmed to a chunk boundary, hadooprpc.c:832-840),
    #    all-zero (ftruncate/NULL buffer, hadooprpc.c:694-697), all-0xFF,
    #    and an unaligned start (crc32c.c:241-247 / 85-88).
    cases = []
    rng_seed = 1000
    for bpc in [512, 1024, 4096, 100, 1536]:
        shapes = [
            ("xorshift", 65536, 0), ("xorshift", 65536 - 100, 0), ("xorshift", bpc - 1, 0), ("xorshift", 3, 0),
            ("xorshift", 1, 0), ("zero", 65536, 0), ("ff", 65536, 0), ("xorshift", 65536, 3),
            ("xorshift", 5 * bpc + 17, 13), ("ramp", 8192, 0),
        ]
        for kind, n, align in shapes:
            rng_seed += 1
            buf = fill(kind, n + align, rng_seed)[align:]
            pk = np.zeros(1, dtype=oracle.PACKET_DTYPE)
            pk["len"] = n
            pk["bpc"] = bpc
            exp = ref.batch(buf, pk, (n + bpc - 1) // bpc)
            cases.append({"bpc": bpc, "kind": kind, "seed": rng_seed, "len": n, "skip": align,
                          "crcs": [hx(int(v)) for v in exp]})
    with open(os.path.join(OUT, "packets.json"), "w") as f:
        json.dump({"payload": "bytes [skip, skip+len) of fill(kind, len+skip, seed); see make_golden.fill",
                   "cases": cases}, f, indent=0)

    # 3. Whole-batch digests for the BASELINE.json configs.  Payload is one
    #    xorshift64 stream over the whole batch buffer.
    batches = []
    specs = [
        ("c1_one_packet", oracle.uniform_packets(1)),
        ("c3_one_block_4MiB", oracle.uniform_packets(64)),
        ("c5_mixed_bpc_96", oracle.mixed_packets(96)),
        ("c2_4096_packets", oracle.uniform_packets(4096)),
        ("c5_mixed_bpc_4096", oracle.mixed_packets(4096)),
        ("ragged_tail_257", oracle.uniform_packets(257, pkt_len=65436, bpc=512, stride=65536)),
        # config 4: a 128 MiB file = 32 blocks x 64 packets, checksums in file order
        ("c4_file_128MiB", oracle.uniform_packets(2048)),
        # config 2 with bytesPerChecksum 1536 (general tiles + 1024-byte tails)
        ("c2_bpc1536", oracle.uniform_packets(4096, bpc=1536)),
    ]
    for name, pk in specs:
        nbytes = int((pk["payload_off"] + pk["len"]).max())
        payload = fill("xorshift", nbytes, oracle.SEED)
        nout = oracle.total_checksums(pk)
        exp = ref.batch(payload, pk, nout)
        batches.append({
            "name": name, "seed": oracle.SEED, "payload_bytes": nbytes, "nchecksums": nout,
            "packets": {"count": int(pk.size), "len": [int(x) for x in np.unique(pk["len"])],
                        "bpc_cycle": [int(x) for x in pk["bpc"][:3]],
                        "layout": "mixed_packets" if name.startswith("c5") else "uniform_packets",
                        "bpc": int(pk["bpc"][0]),
                        "stride": int(pk["payload_off"][1]) if pk.size > 1 else 0},
            "sha256_le": hashlib.sha256(exp.astype("<u4").tobytes()).hexdigest(),
            "head": [hx(int(v)) for v in exp[:8]], "tail": [hx(int(v)) for v in exp[-8:]],
        })
    with open(os.path.join(OUT, "batches.json"), "w") as f:
        json.dump(batches, f, indent=1)
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
