"""Diagnostic: is config 3's per-launch time host-bound?  Times back-to-back
plan.exec launches issued from Python against the same launches replayed from
a captured graph, and the host's issue time."""
import sys, os, time, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from bench import load_package
h = load_package()
from hdfs_crc32c_amd.workloads import config_packets
res = {}
for cfg in ("c3", "p16", "p256"):
    pk, _ = config_packets(cfg)
    extent = int((pk["payload_off"] + pk["len"]).max())
    n = h.total_checksums(pk)
    ctx = h.Context(0)
    plan = ctx.plan(pk)
    bufs = [torch.randint(0, 256, (extent,), dtype=torch.uint8, device="cuda") for _ in range(4)]
    outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(4)]
    s = torch.cuda.Stream()
    K = 2000
    with torch.cuda.stream(s):
        for i in range(200):
            plan.exec(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        t0 = time.perf_counter()
        for i in range(K):
            plan.exec(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), s.cuda_stream)
        t1 = time.perf_counter()
        e1.record(s)
        torch.cuda.synchronize()
        py_us = e0.elapsed_time(e1) / K * 1e3
        issue_us = (t1 - t0) / K * 1e6
        g = torch.cuda.CUDAGraph()
        G = 100
        with torch.cuda.graph(g, stream=s):
            for i in range(G):
                plan.exec(bufs[i % 4].data_ptr(), outs[i % 4].data_ptr(), s.cuda_stream)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0.record(s)
        R = 20
        for _ in range(R):
            g.replay()
        e1.record(s)
        torch.cuda.synchronize()
        graph_us = e0.elapsed_time(e1) / (R * G) * 1e3
    got = outs[0].cpu().numpy().view(np.uint32)
    res[cfg] = {"python_loop_us": round(py_us, 2), "host_issue_us": round(issue_us, 2), "graph_us": round(graph_us, 2)}
    print(cfg, res[cfg], flush=True)
    plan.close(); ctx.close()
print(json.dumps(res))
