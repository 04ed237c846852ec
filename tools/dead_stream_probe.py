#!/usr/bin/env python3
"""What HIP does with a stream the caller has already destroyed: each call in
its own child process (a segfault there is contained), one JSON line each.
Also: does hipStreamDestroy wait for work still queued on the stream?"""
import ctypes
import json
import subprocess
import sys

CALLS = ["hipStreamQuery", "hipStreamIsCapturing", "hipEventRecord", "hipStreamWaitEvent", "hipStreamSynchronize"]


def child(call: str) -> None:
    hip = ctypes.CDLL("libamdhip64.so")
    s = ctypes.c_void_p()
    hip.hipSetDevice(0)
    hip.hipStreamCreate(ctypes.byref(s))
    hip.hipStreamDestroy(s)
    e = ctypes.c_void_p()
    hip.hipEventCreateWithFlags(ctypes.byref(e), 2)
    other = ctypes.c_void_p()
    if call == "hipStreamQuery":
        rc = hip.hipStreamQuery(s)
    elif call == "hipStreamIsCapturing":
        st = ctypes.c_int(0)
        rc = hip.hipStreamIsCapturing(s, ctypes.byref(st))
    elif call == "hipEventRecord":
        rc = hip.hipEventRecord(e, s)
    elif call == "hipStreamWaitEvent":
        hip.hipEventRecord(e, None)
        rc = hip.hipStreamWaitEvent(s, e, 0)
    else:
        rc = hip.hipStreamSynchronize(s)
    hip.hipStreamCreate(ctypes.byref(other))
    print(json.dumps({"call": call, "rc": rc, "handle_reused": other.value == s.value}), flush=True)


def destroy_waits() -> None:
    """A long kernel-free wait queued on a stream (hipStreamWaitEvent on an
    event recorded behind a 200 ms host sleep would need a host callback; use
    a big memset instead), then destroy: does destroy return before it ends?"""
    import time

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipSetDevice(0)
    s = ctypes.c_void_p()
    hip.hipStreamCreate(ctypes.byref(s))
    p = ctypes.c_void_p()
    n = 8 << 30
    hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n))
    ev = ctypes.c_void_p()
    hip.hipEventCreateWithFlags(ctypes.byref(ev), 2)
    for _ in range(20):
        hip.hipMemsetAsync(p, 1, ctypes.c_size_t(n), s)
    hip.hipEventRecord(ev, s)
    t0 = time.perf_counter()
    hip.hipStreamDestroy(s)
    t1 = time.perf_counter()
    q = hip.hipEventQuery(ev)
    hip.hipEventSynchronize(ev)
    t2 = time.perf_counter()
    print(json.dumps({"destroy_ms": round((t1 - t0) * 1e3, 3), "event_query_after_destroy": q,
                      "work_left_after_destroy_ms": round((t2 - t1) * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "destroy":
        destroy_waits()
    elif len(sys.argv) > 1:
        child(sys.argv[1])
    else:
        for c in CALLS:
            r = subprocess.run([sys.executable, __file__, c], capture_output=True, text=True, timeout=60)
            line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else ""
            print(line if line else json.dumps({"call": c, "returncode": r.returncode}), flush=True)
        r = subprocess.run([sys.executable, __file__, "destroy"], capture_output=True, text=True, timeout=120)
        print(r.stdout.strip() or json.dumps({"destroy": "rc %d" % r.returncode, "err": r.stderr[-300:]}), flush=True)
