"""N>1 path on CPU: world-size-2 gloo runs of the sharding and the counter
all-reduce that bench.py uses on GPUs (RCCL there), with the oracle as the
per-rank parser (test infrastructure; the GPU path is covered by -m gpu)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import logparser_amd as lpa
from logparser_amd.shard import line_aligned_ranges, max_over_ranks, reduce_counters


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_line_aligned_ranges_partition_lines():
    data = lpa.synth_combined(4, 0, 5000)
    for parts in (1, 2, 3, 8, 13):
        rs = line_aligned_ranges(data, parts)
        assert rs[0][0] == 0 and rs[-1][1] == len(data)
        for (a, b), (c, _) in zip(rs, rs[1:]):
            assert b == c
        got = []
        for a, b in rs:
            assert a == 0 or data[a - 1:a] == b"\n"
            got += data[a:b].split(b"\n")[:-1] if b > a else []
        assert got == data.split(b"\n")[:-1]


def test_line_aligned_ranges_edge_cases():
    assert line_aligned_ranges(b"", 2) == [(0, 0), (0, 0)]
    assert line_aligned_ranges(b"abc", 3) == [(0, 3), (3, 3), (3, 3)]  # one unterminated line
    d = b"a\nbb\nccc\n"
    rs = line_aligned_ranges(d, 4)
    assert sum(d[a:b].count(b"\n") for a, b in rs) == 3


def _worker(rank, world, port, data, fields, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle_lib

    a, b = line_aligned_ranges(data, world)[rank]
    o = oracle_lib.Oracle("combined", fields)
    c = np.zeros(4, dtype=np.int64)
    for line in data[a:b].split(b"\n")[:-1]:
        st, _ = o.parse_raw(line)
        c[0] += 1
        c[1 + min(st, 2)] += 1
    t = reduce_counters(torch.from_numpy(c))
    m = max_over_ranks(float(rank + 1))
    out[rank] = t.tolist() + [m]
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_counters(oracle):
    fields = ["IP:connection.client.host", "TIME.EPOCH:request.receive.time.epoch",
              "STRING:request.firstline.uri.query.*"]
    lines = lpa.synth_combined(6, 0, 3000).split(b"\n")[:-1]
    lines[10] = b"garbage line"
    lines[2000] = lines[2000][:40]
    data = b"\n".join(lines) + b"\n"
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), data, fields, out), nprocs=2, join=True)
    o = oracle.Oracle("combined", fields)
    ref = [0, 0, 0, 0]
    for line in lines:
        st, _ = o.parse_raw(line)
        ref[0] += 1
        ref[1 + min(st, 2)] += 1
    assert out[0][:4] == ref and out[1][:4] == ref
    assert ref[2] == 2
    assert out[0][4] == out[1][4] == 2.0


def test_line_aligned_ranges_cr_terminators():
    import corpora
    lines = lpa.synth_combined(7, 0, 3000).split(b"\n")[:-1]
    data = corpora.crlf_join(lines, 3)
    for parts in (2, 3, 7):
        got = []
        for a, b in line_aligned_ranges(data, parts):
            got += corpora.split_hadoop(data[a:b])
        assert got == lines
    from logparser_amd.shard import count_terminators
    assert count_terminators(np.frombuffer(b"a\r\nb\rc\n\r\r\n", dtype=np.uint8)) == 5


def _stream_split_local(chunks, rank, world, group=None):
    """stream_split over numpy home chunks (the CPU stand-in of device buffers)"""
    from logparser_amd.shard import count_terminators, stream_split
    import corpora
    mine = np.frombuffer(chunks[rank], dtype=np.uint8)
    n_lines = len(corpora.split_hadoop(chunks[rank]))
    return stream_split(len(mine), n_lines, lambda off, n: mine[off:off + n],
                        lambda a, b: count_terminators(mine[a:b]), group=group)


def test_stream_split_matches_line_aligned_ranges_single_process():
    """stream_split's cuts == line_aligned_ranges on the concatenated stream
    (the collectives replaced by the loop over ranks the all-reduce merges)"""
    import corpora
    lines = lpa.synth_combined(8, 0, 4000).split(b"\n")[:-1]
    for world, sizes in ((2, [2100, 1900]), (3, [1000, 1500, 1500]), (4, [50, 3000, 900, 50])):
        data_lines, chunks, k = lines, [], 0
        for sz in sizes:
            part = data_lines[k:k + sz]
            k += sz
            chunks.append(corpora.crlf_join(part, k) + (b"\r\n" if k < len(lines) else b""))
        stream = b"".join(chunks)
        want = line_aligned_ranges(stream, world)
        # emulate the all-gather / all-reduce: every rank resolves its own cuts
        g = np.cumsum([0] + [len(c) for c in chunks])
        gl = np.cumsum([0] + [len(corpora.split_hadoop(c)) for c in chunks])
        pos = [0] * (world + 1)
        first = [0] * (world + 1)
        for r in range(world):
            f, p = _split_as_rank(chunks, r, world)
            for j in range(1, world):
                s = (j * len(stream)) // world
                if g[r] <= s < g[r + 1]:
                    pos[j], first[j] = p[j], f[j]
        pos[world], first[world] = len(stream), int(gl[-1])
        assert [(pos[j], max(pos[j], pos[j + 1])) for j in range(world)] == want
        for j in range(world):
            assert first[j] == len(corpora.split_hadoop(stream[:pos[j]]))


def _split_as_rank(chunks, rank, world):
    """one rank's view of stream_split without a process group: the all_gather
    and the all-reduce are replaced by their results over the given chunks"""
    import corpora
    from unittest import mock
    import torch.distributed as dist
    sizes = [torch.tensor([len(c), len(corpora.split_hadoop(c))]) for c in chunks]

    def all_gather(out, t, group=None):
        for i, v in enumerate(sizes):
            out[i].copy_(v)

    with mock.patch.object(dist, "is_initialized", return_value=True), \
            mock.patch.object(dist, "get_world_size", return_value=world), \
            mock.patch.object(dist, "get_rank", return_value=rank), \
            mock.patch.object(dist, "all_gather", side_effect=all_gather), \
            mock.patch.object(dist, "all_reduce", side_effect=lambda *a, **k: None):
        return _stream_split_local(chunks, rank, world)


def _split_worker(rank, world, port, chunks, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out[rank] = _stream_split_local(chunks, rank, world)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_stream_split():
    """world-size-2 gloo: all_gather of chunk sizes / line counts, all-reduce of
    the cuts; both ranks agree, and the splits are line_aligned_ranges' with
    global line numbers"""
    import corpora
    lines = lpa.synth_combined(9, 0, 3000).split(b"\n")[:-1]
    chunks = [corpora.crlf_join(lines[:1700], 1) + b"\r\n", corpora.crlf_join(lines[1700:], 2)]
    stream = b"".join(chunks)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_split_worker, args=(2, _free_port(), chunks, out), nprocs=2, join=True)
    assert out[0] == out[1]
    first, pos = out[0]
    assert [(pos[0], pos[1]), (pos[1], pos[2])] == line_aligned_ranges(stream, 2)
    assert first == [0, len(corpora.split_hadoop(stream[:pos[1]])), 3000]


def _bench_split_worker(rank, world, port, L, out, wl=2, batch_bytes=0):
    """bench.py's split of one synthetic stream (CPU tensors for the HBM buffer)"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    home = lpa.synth(wl, bench.SEEDS[wl], rank * L, L)
    front = 1 << 20
    buf = torch.zeros(front + len(home) + (1 << 20), dtype=torch.uint8)
    buf[front:front + len(home)] = torch.frombuffer(bytearray(home), dtype=torch.uint8)
    (off, nb), first, cuts = bench.split_stream(lpa, torch, buf, front, len(home), wl, L, rank, None)
    pieces = bench.newline_batches(buf, off, nb, batch_bytes)
    out[rank] = (bytes(buf[off:off + nb].numpy()), first, cuts, [bytes(buf[a:a + n].numpy()) for a, n in pieces])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_bench_stream_split_gloo():
    """bench.py --gpus N on one stream: each rank's batch is exactly its
    Hadoop split of the concatenated stream, and the splits tile it"""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    L, world = 1500, 3
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bench_split_worker, args=(world, _free_port(), L, out), nprocs=world, join=True)
    stream = lpa.synth(2, 20261015, 0, world * L)
    want = line_aligned_ranges(stream, world)
    assert out[0][1] == out[1][1] == out[2][1]
    for r in range(world):
        a, b = want[r]
        assert out[r][0] == stream[a:b], r
        assert out[r][2][r] == a
    assert out[0][1][-1] == world * L


@pytest.mark.timeout(600)
def test_bench_stream_split_config5_gloo(oracle):
    """bench.py --gpus 2 --workload 5: one config-5 stream in Hadoop splits,
    each split cut into newline-aligned batches.  The splits and batches tile
    the stream, and (the LogFormats being mutually exclusive) every line's
    result from a parser that starts at a split or batch boundary equals the
    result of one parser over the whole stream (the sticky format state at a
    boundary changes nothing) -- checked with the oracle."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import corpora
    oracle_lib = oracle
    L, world = 1200, 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bench_split_worker, args=(world, _free_port(), L, out, 5, 64 << 10), nprocs=world, join=True)
    stream = lpa.synth(5, bench.SEEDS[5], 0, world * L)
    want = line_aligned_ranges(stream, world)
    for r in range(world):
        a, b = want[r]
        assert out[r][0] == stream[a:b], r
        assert b"".join(out[r][3]) == out[r][0] and len(out[r][3]) > 1, r
        assert all(p.endswith(b"\n") for p in out[r][3][:-1]), r
    assert out[0][1][-1] == world * L
    fmt = lpa.SYNTH_FORMATS[5]
    fields = [f for f in oracle_lib.possible_paths(fmt) if "firstline" in f or "status" in f or "epoch" in f][:24]
    whole = oracle_lib.Oracle(fmt, fields)
    ref = [whole.parse_raw(x) for x in corpora.split_hadoop(stream)]
    got = []
    for r in range(world):
        for piece in out[r][3]:
            o = oracle_lib.Oracle(fmt, fields)  # a fresh sticky state at every boundary
            got += [o.parse_raw(x) for x in corpora.split_hadoop(piece)]
    assert len(got) == len(ref) == world * L
    assert got == ref
    assert sum(1 for st, _ in ref if st == oracle_lib.OK) > 0.9 * len(ref)


def test_bench_gpus_flag_launches_ranks():
    """`python bench.py --gpus N` (WORLD_SIZE unset) starts N rank processes
    itself (torch.distributed.run as a child process, before any GPU call);
    LP_BENCH_DRYRUN stops each rank right after its process group is up, so
    the launcher path runs on CPU (gloo) up to its pre-GPU point."""
    import json
    import re
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["LP_BENCH_DRYRUN"] = "1"
    for n in (1, 3):
        p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n)], env=env,
                           capture_output=True, text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-2000:]
        # the ranks share one stdout: pick the objects out wherever they landed
        lines = [json.loads(x) for x in re.findall(r'\{"dryrun"[^{}]*\}', p.stdout)]
        assert sorted(x["rank"] for x in lines) == list(range(n)), p.stdout
        for x in lines:
            assert x["world_size"] == n and x["gpus"] == n
            assert x["backend"] == ("gloo" if n > 1 else None)
    # a driver-style launch whose WORLD_SIZE disagrees with --gpus fails loudly
    env2 = dict(env, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"], env=env2,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=2" in (p.stderr + p.stdout)
