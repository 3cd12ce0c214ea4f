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
