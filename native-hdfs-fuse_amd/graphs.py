"""Rank-consistent HIP-graph capture of a step that holds collective calls.

A multi-GPU step (crc32c_multi_plan_exec: the shard launches plus ONE RCCL
group of send / receive calls, csrc/crc32c_multi.hip) must be captured into a
graph on every rank or on none: a rank that replays a graph and a rank that
issues the same step from the host still post the same RCCL calls in the same
order, but a rank whose capture failed part-way through an RCCL group may
have left that group half-posted in its communicator, and its peers would
then wait on transfers it never makes.  So:

1. every rank first captures a probe with no collective in it (the shard's
   plan launch alone); if any rank's probe fails, no rank captures the real
   step and no RCCL call has been recorded anywhere;
2. every rank captures the step; the ranks agree on the outcome with a MIN
   all-reduce;
3. if any rank failed, every rank drops what it captured and runs
   ``on_abandon`` -- the caller rebuilds the communicator (a new id, a new
   ``crc32c_multi`` handle), so no half-posted group survives -- and every
   rank then issues its steps from the host.

``inject_fail`` makes this rank's step capture fail (bench.py:
``BENCH_CAPTURE_FAIL_RANK``), so the fallback can be tested on purpose
(tests/test_distributed.py runs it over gloo on the CPU).
"""
from __future__ import annotations


def agree(ok: bool, world: int, device=None) -> bool:
    """True on every rank iff ``ok`` on every rank (MIN all-reduce)."""
    if world <= 1:
        return bool(ok)
    import torch
    import torch.distributed as dist

    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def capture_agreed(capture, world: int, device=None, probe=None, on_abandon=None, inject_fail: bool = False):
    """Run ``probe()`` then ``capture()`` (each raises ``RuntimeError`` on a
    failed capture) with the ranks agreeing after each.  Returns
    ``(captured, error)``: ``captured`` is what ``capture()`` returned when
    every rank succeeded, else None on every rank; ``error`` says why (this
    rank's own error, or that another rank failed).  ``on_abandon()`` runs on
    every rank (collectively) when the step capture failed on any rank."""
    err = None
    if probe is not None:
        try:
            probe()
        except RuntimeError as e:
            err = "probe capture: %s" % str(e)[:200]
        if not agree(err is None, world, device):
            return None, err or "another rank's probe capture failed"
    got = None
    try:
        if inject_fail:
            raise RuntimeError("injected step-capture failure (BENCH_CAPTURE_FAIL_RANK)")
        got = capture()
    except RuntimeError as e:
        err = str(e)[:200]
    if agree(err is None, world, device):
        return got, None
    got = None
    if on_abandon is not None:
        on_abandon()
    return None, err or "another rank's step capture failed"
