"""The library's host-only sources (crc_math.cpp, cpu_crc32c.cpp, plan.cpp, frames.cpp,
framing.cpp) built with AddressSanitizer + UndefinedBehaviorSanitizer and
driven by tests/sanitize/host_asan.cpp over randomized inputs held in
exactly-sized heap blocks, checked against the oracle restatement.  CPU only
(GPU sanitizers are not available on the pool)."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "native-hdfs-fuse_amd", "csrc")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no host compiler")
def test_host_sources_under_asan_ubsan(tmp_path):
    oracle_o = str(tmp_path / "oracle.o")
    exe = str(tmp_path / "host_asan")
    subprocess.run(["gcc", *SAN, "-c", os.path.join(ROOT, "oracle", "crc32c_oracle.c"), "-o", oracle_o],
                   check=True)
    srcs = [os.path.join(CSRC, f) for f in ("errors.cpp", "crc_math.cpp", "cpu_crc32c.cpp", "plan.cpp", "framing.cpp", "frames.cpp")]
    subprocess.run(["g++", *SAN, "-std=c++17", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
                    "-I/opt/rocm/include", os.path.join(ROOT, "tests", "sanitize", "host_asan.cpp"), *srcs,
                    oracle_o, "-lpthread", "-o", exe], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host sanitizer run clean" in r.stdout


TSAN = ["-fsanitize=thread", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no host compiler")
def test_host_threads_under_tsan(tmp_path):
    """ThreadSanitizer over the host runtime's threaded code: the staging-copy
    workers and their piece hand-off (host_copy.h, crc32c_batch_host's
    pageable path), the lazily initialised CPU dispatcher and tables under 12
    concurrent callers (libfuse's worker threads), concurrent plan building,
    framing and frame parsing (tests/sanitize/host_tsan.cpp)."""
    oracle_o = str(tmp_path / "oracle.o")
    exe = str(tmp_path / "host_tsan")
    subprocess.run(["gcc", *TSAN, "-fPIC", "-c", os.path.join(ROOT, "oracle", "crc32c_oracle.c"), "-o", oracle_o],
                   check=True)
    srcs = [os.path.join(CSRC, f) for f in ("errors.cpp", "crc_math.cpp", "cpu_crc32c.cpp", "plan.cpp", "framing.cpp", "frames.cpp")]
    subprocess.run(["g++", *TSAN, "-std=c++17", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
                    "-I/opt/rocm/include", os.path.join(ROOT, "tests", "sanitize", "host_tsan.cpp"), *srcs,
                    oracle_o, "-lpthread", "-o", exe], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "host tsan run clean" in r.stdout and "WARNING: ThreadSanitizer" not in r.stderr
