"""Shared fixtures.  CPU tests (-m "not gpu") cover the oracle against the
golden vectors, the host logic of the library and a bit-level model of the
kernel; @pytest.mark.gpu tests are the parity tests proper and call the HIP
path through the C ABI."""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
PKG_DIR = os.path.join(ROOT, "native-hdfs-fuse_amd")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU; parity tests of the HIP path")


def load_package():
    """Import native-hdfs-fuse_amd/ (a directory name Python cannot import by name)."""
    if "hdfs_crc32c_amd" in sys.modules:
        return sys.modules["hdfs_crc32c_amd"]
    spec = importlib.util.spec_from_file_location("hdfs_crc32c_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["hdfs_crc32c_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def hdfs():
    mod = load_package()
    if not os.path.exists(mod.LIB_PATH):
        mod.build()
    mod.lib()
    return mod


@pytest.fixture(scope="session")
def orc():
    import oracle

    oracle.build()
    return oracle.Oracle()


@pytest.fixture(scope="session")
def golden():
    out = {}
    for name in ("known_answers", "packets", "batches"):
        with open(os.path.join(GOLDEN, name + ".json")) as f:
            out[name] = json.load(f)
    return out


def golden_fill(kind: str, n: int, seed: int) -> np.ndarray:
    import oracle

    if kind == "xorshift":
        return oracle.xorshift64_bytes(n, seed)
    if kind == "zero":
        return np.zeros(n, np.uint8)
    if kind == "ff":
        return np.full(n, 0xFF, np.uint8)
    if kind == "ramp":
        return (np.arange(n) & 0xFF).astype(np.uint8)
    raise ValueError(kind)


def golden_batch_packets(spec: dict) -> np.ndarray:
    import oracle

    p = spec["packets"]
    if p["layout"] == "mixed_packets":
        return oracle.mixed_packets(p["count"], pkt_len=p["len"][0])
    stride = p["stride"] or p["len"][0]
    return oracle.uniform_packets(p["count"], pkt_len=p["len"][0], bpc=p["bpc_cycle"][0], stride=stride)


@pytest.fixture(scope="session")
def gpu_ctx(hdfs):
    return hdfs.Context(0)
