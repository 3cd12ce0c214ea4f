"""Multi-GPU partitioning of one log byte stream.

Lines are independent, so G GPUs each parse a newline-aligned byte range and
only counters are combined (RCCL all-reduce; `reduce_counters`).  The ranges
follow Hadoop LineRecordReader split semantics, which the reference's input
format relies on (ApacheHttpdLogfileRecordReader.java:57,115): the stream is
cut at G equal byte offsets s_k; a line whose first byte lies in
(s_k, s_{k+1}] belongs to split k (split 0 also owns the line at byte 0), so a
split skips the partial line at its start and finishes the line that crosses
its end.  Every line lands in exactly one split.  Line terminators are
LineReader's: '\n', '\r', or "\r\n" (one terminator).

`line_aligned_ranges` cuts a buffer one process holds; `stream_split` cuts a
stream whose consecutive, line-aligned pieces ("home chunks") are held by the
ranks, one each: an all_gather of the chunk sizes and line counts places the
cuts, each rank resolves the cuts that fall in its own chunk, and an
all-reduce shares them -- the global line number of every split's first line
comes out of the same exchange.
"""
import numpy as np


def _term_end(buf, t):
    """end of the terminator at t ("\r\n" is one)"""
    return t + 2 if buf[t] == 13 and t + 1 < len(buf) and buf[t + 1] == 10 else t + 1


def _after_newline(buf, pos):
    """Start of the first line that begins after pos: just past the first
    terminator at or after pos (len(buf) if none).  A '\r' at pos - 1 with
    '\n' at pos is one terminator ending at pos + 1."""
    n = len(buf)
    if pos >= n:
        return n
    hit = np.flatnonzero((buf[pos:] == 10) | (buf[pos:] == 13))
    if hit.size == 0:
        return n
    return _term_end(buf, pos + int(hit[0]))


def count_terminators(buf):
    """Hadoop line terminators in buf: '\n' plus every '\r' not followed by '\n'"""
    buf = np.asarray(buf)
    lf = int(np.count_nonzero(buf == 10))
    cr = buf == 13
    if not cr.any():
        return lf
    crlf = int(np.count_nonzero(cr[:-1] & (buf[1:] == 10)))
    return lf + int(np.count_nonzero(cr)) - crlf


def line_aligned_ranges(data, parts):
    """[(start, end)) byte ranges, one per split, covering data exactly."""
    buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) else data
    n = len(buf)
    cuts = [0] + [_after_newline(buf, (n * k) // parts) for k in range(1, parts)] + [n]
    return [(cuts[k], max(cuts[k], cuts[k + 1])) for k in range(parts)]


def stream_split(chunk_bytes, chunk_lines, window, count, group=None, device=None):
    """Hadoop splits of a stream held as one line-aligned home chunk per rank
    (rank order = stream order; every chunk but the last ends with a line
    terminator).

    chunk_bytes / chunk_lines: this rank's chunk size and line count.
    window(off, n) -> the chunk's bytes [off, off + n) (a numpy uint8 array;
    fewer at the chunk's end); count(a, b) -> Hadoop terminators in the
    chunk's bytes [a, b).  Collectives: one all_gather of (bytes, lines) and
    one all-reduce (max) of the cuts.

    Returns (first, pos): for every split k of the world, its first line's
    global number first[k] and global byte offset pos[k]; first[W] / pos[W]
    are the stream's line count / size.  Split k is lines [first[k],
    first[k+1]), bytes [pos[k], pos[k+1])."""
    import torch
    import torch.distributed as dist

    dist_on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if dist_on else 1
    rank = dist.get_rank(group) if dist_on else 0
    mine = torch.tensor([int(chunk_bytes), int(chunk_lines)], dtype=torch.int64, device=device)
    if world > 1:
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine, group=group)
        sizes = [(int(v[0]), int(v[1])) for v in allv]
    else:
        sizes = [(int(chunk_bytes), int(chunk_lines))]
    g_byte = np.cumsum([0] + [b for b, _ in sizes]).tolist()
    g_line = np.cumsum([0] + [l for _, l in sizes]).tolist()
    total_b, total_l = g_byte[-1], g_line[-1]
    # cut k (1 <= k < W): the first line starting after s_k = k * B / W
    cuts = torch.full((2 * world,), -1, dtype=torch.int64, device=device)
    for k in range(1, world):
        s = (k * total_b) // world
        if not (g_byte[rank] <= s < g_byte[rank + 1]):
            continue
        off = s - g_byte[rank]
        p, step = None, 1 << 16
        while p is None:
            w = np.asarray(window(off, step))
            hit = np.flatnonzero((w == 10) | (w == 13))
            if hit.size:
                t = int(hit[0])
                if w[t] == 13 and t + 1 >= len(w) and off + len(w) < chunk_bytes:
                    step *= 2  # a '\r' at the window's end: see whether '\n' follows
                    continue
                p = off + _term_end(w, t)
            elif off + len(w) >= chunk_bytes:
                p = chunk_bytes  # an unterminated last line runs to the end
            else:
                step *= 2
        # p == chunk end: the next chunk's first line (home chunks are line-aligned)
        cuts[2 * k] = g_line[rank + 1] if p >= chunk_bytes else g_line[rank] + int(count(0, p))
        cuts[2 * k + 1] = g_byte[rank] + p
    if world > 1:
        dist.all_reduce(cuts, op=dist.ReduceOp.MAX, group=group)
    first = [0] + [int(cuts[2 * k]) for k in range(1, world)] + [total_l]
    pos = [0] + [int(cuts[2 * k + 1]) for k in range(1, world)] + [total_b]
    for k in range(1, world + 1):  # empty splits (cuts past the last line start) stay empty
        first[k] = max(first[k], first[k - 1])
        pos[k] = max(pos[k], pos[k - 1])
    return first, pos


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
