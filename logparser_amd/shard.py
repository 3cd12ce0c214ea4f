"""Multi-GPU partitioning of one log byte stream.

Lines are independent, so G GPUs each parse a newline-aligned byte range and
only the counters are combined (RCCL all-reduce; `reduce_counters`).  The
ranges follow Hadoop LineRecordReader split semantics, which the reference's
input format relies on (ApacheHttpdLogfileRecordReader.java:57,115): the
stream is cut at G equal byte offsets s_k; a line whose first byte lies in
(s_k, s_{k+1}] belongs to split k (split 0 also owns the line at byte 0), so a
split skips the partial line at its start and finishes the line that crosses
its end.  Every line lands in exactly one split.
"""
import numpy as np


def _after_newline(buf, pos):
    """Index just after the first '\\n' at or after pos (len(buf) if none)."""
    n = len(buf)
    if pos >= n:
        return n
    hit = np.flatnonzero(buf[pos:] == 10)
    return n if hit.size == 0 else pos + int(hit[0]) + 1


def line_aligned_ranges(data, parts):
    """[(start, end)) byte ranges, one per split, covering data exactly."""
    buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) else data
    n = len(buf)
    cuts = [0] + [_after_newline(buf, (n * k) // parts) for k in range(1, parts)] + [n]
    return [(cuts[k], max(cuts[k], cuts[k + 1])) for k in range(parts)]


def reduce_counters(counters, group=None):
    """All-reduce (sum) a tensor of per-rank line counters [lines, ok, bad,
    fallback]; RCCL on GPUs, gloo in the CPU tests."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    return counters


def max_over_ranks(value, device=None, group=None):
    """Max of a float over ranks (the benchmark's timed region)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
