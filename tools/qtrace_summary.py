#!/usr/bin/env python3
"""Summarise a block-queue trace (HDFS_CRC32C_QUEUE_TRACE, crc32c_blocks.hip).

Per flush: fill = issue start - first submit; issue = the launch call;
latency = completion seen - issue end; service = completion seen -
max(previous completion seen, issue end) (~ the GPU time of a flush queued
behind another); interval = between successive issue ends.  Medians and
means in us, per queue (a trace file holds one block of lines per queue,
ended by {"end": 1})."""
import json
import statistics
import sys


def summarise(recs):
    out = {"flushes": len(recs)}
    if not recs:
        return out
    f = lambda k: [r[k] / 1e3 for r in recs]
    fill = [(r["issue0"] - r["first"]) / 1e3 for r in recs]
    issue = [(r["issue1"] - r["issue0"]) / 1e3 for r in recs]
    lat = [(r["done"] - r["issue1"]) / 1e3 for r in recs if r["done"]]
    serv, inter = [], []
    for a, b in zip(recs, recs[1:]):
        if a["done"] and b["done"]:
            serv.append((b["done"] - max(a["done"], b["issue1"])) / 1e3)
        inter.append((b["issue1"] - a["issue1"]) / 1e3)
    for name, v in (("fill", fill), ("issue", issue), ("latency", lat), ("service", serv), ("interval", inter)):
        if v:
            out[name] = {"median": round(statistics.median(v), 2), "mean": round(statistics.fmean(v), 2)}
    out["blocks_per_flush"] = round(statistics.fmean(r["nblocks"] for r in recs), 2)
    out["inflight_before"] = round(statistics.fmean(r["inflight_before"] for r in recs), 2)
    span = (recs[-1]["done"] - recs[0]["issue0"]) / 1e3 if recs[-1]["done"] else None
    if span:
        out["us_per_block"] = round(span / sum(r["nblocks"] for r in recs), 3)
    return out


def main():
    cur = []
    for line in open(sys.argv[1]):
        r = json.loads(line)
        if "end" in r:
            print(json.dumps(summarise(cur)))
            cur = []
        else:
            cur.append(r)


if __name__ == "__main__":
    main()
