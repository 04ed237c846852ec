import sys, time, numpy as np
sys.path.insert(0, '.')
from bench import load_package
h = load_package()
from hdfs_crc32c_amd.workloads import synthetic_bytes
pkt = synthetic_bytes(65536, 5)
h.chunks(pkt, 512)
for name, f in (("crc32c_chunks (GPU, default ctx)", lambda: h.chunks(pkt, 512)), ("crc32c_chunks_cpu", lambda: h.chunks_cpu(pkt, 512))):
    t0 = time.perf_counter()
    for _ in range(300):
        f()
    print(name, "%.1f us per 64 KiB packet" % ((time.perf_counter() - t0) / 300 * 1e6))
assert np.array_equal(h.chunks(pkt, 512), h.chunks_cpu(pkt, 512))
