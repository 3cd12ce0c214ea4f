"""Benchmark of the logparser hot path on MI355X (BASELINE.json config 2).

One step = one lp_parse_batch over the rank's whole input, resident in HBM:
newline index + match/dissect every line with all 123 'combined' paths
requested (incl. epoch timestamp, first line, URI parts, query parameters),
then an RCCL all-reduce of the line counters (world > 1).

Default workload: 100M synthetic 'combined' lines per GPU (~25 GB, seed
20261015), weak scaling over GPUs (each rank parses its own 100M lines).
Prints ONE JSON line on rank 0.  --workload 3 / 4 runs BASELINE.json configs
3 (strftime timestamps, 5 % malformed lines) and 4 (NGINX upstream log
format) the same way, for the records in DESIGN.md; the headline is config 2.
--workload 5 is config 5: a mixed-format corpus (40 % 'combined', 30 % config-4
NGINX, 30 % 'common' lines) parsed by one three-format handle (sticky active
format on the device), streamed through it in ~1 GiB newline-aligned batches
so the routing state is carried across batches; it also reports the
PCIe-inclusive rate of host-resident batches (H2D copy inside the call).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--lines L] [--workload 2|3|4|5]
"""
import argparse
import concurrent.futures as cf
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SEEDS = {2: 20261015, 3: 20261016, 4: 20261017, 5: 20261018}
WORKLOAD_NAMES = {2: "config 2: %d synthetic 'combined' lines",
                  3: "config 3: %d synthetic 'combinedio' + %%{%%d/%%b/%%Y %%T}t.%%{msec_frac}t lines (5%% malformed)",
                  4: "config 4: %d synthetic NGINX '$request_time $upstream_response_time $pipe' lines",
                  5: "config 5: %d synthetic mixed-format lines (40%% 'combined', 30%% NGINX config-4, 30%% 'common')"}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def generate_to_device(lpa, torch, workload, first_line, n_lines, device, chunk=1 << 20, workers=16, batch_bytes=0,
                       front=0):
    """Deterministic synthetic lines [first_line, first_line+n_lines) straight
    into one HBM buffer at offset `front` (host generation in parallel chunks,
    H2D in order).  With batch_bytes, consecutive chunks are grouped into
    batches of about that size, each starting 4 KiB-aligned (as a streaming
    reader's staging buffers would).  Returns (buffer, bytes of lines,
    [(offset, bytes)] batches)."""
    upper = front + n_lines * 320 + (1 << 20)
    dev = torch.empty(upper, dtype=torch.uint8, device=device)
    pos = front
    batches = []
    bstart = front
    starts = list(range(first_line, first_line + n_lines, chunk))
    with cf.ThreadPoolExecutor(max_workers=workers) as ex:
        futs = []
        nxt = 0
        window = 2 * workers
        while nxt < len(starts) and len(futs) < window:
            s = starts[nxt]
            futs.append(ex.submit(lpa.synth, workload, SEEDS[workload], s, min(chunk, first_line + n_lines - s)))
            nxt += 1
        done = 0
        t0 = time.time()
        while futs:
            data = futs.pop(0).result()
            if nxt < len(starts):
                s = starts[nxt]
                futs.append(ex.submit(lpa.synth, workload, SEEDS[workload], s, min(chunk, first_line + n_lines - s)))
                nxt += 1
            if batch_bytes and pos - bstart >= batch_bytes:
                batches.append((bstart, pos - bstart))
                pos = bstart = (pos + 4095) & ~4095
            if pos + len(data) > upper:
                raise RuntimeError("synthetic data larger than the device buffer bound")
            host = torch.frombuffer(bytearray(data), dtype=torch.uint8)
            dev[pos:pos + len(data)].copy_(host)
            pos += len(data)
            done += 1
            if done % 16 == 0:
                log("  generated %d/%d chunks (%.1f GB, %.0f s)" % (done, len(starts), pos / 1e9, time.time() - t0))
    torch.cuda.synchronize()
    batches.append((bstart, pos - bstart))
    return dev, sum(b[1] for b in batches), batches


def device_terminators(torch, x, piece=1 << 30):
    """Hadoop line terminators in the device bytes x ('\n' + lone '\r'), in 1 GiB pieces"""
    n, lf, cr, crlf = x.numel(), 0, 0, 0
    for a in range(0, n, piece):
        v = x[a:min(n, a + piece + 1)]  # one byte of overlap: a "\r\n" across pieces
        body = v[:min(piece, n - a)]
        lf += int((body == 10).sum())
        c = body == 13
        cr += int(c.sum())
        if len(v) > 1:
            crlf += int(((v[:-1] == 13) & (v[1:] == 10))[:len(body)].sum())
    return lf + cr - crlf


def split_stream(lpa, torch, buf, front, nbytes, workload, lines_per_rank, rank, device):
    """This rank's Hadoop split of ONE stream: the ranks' home chunks (lines
    [r L, (r+1) L) of the deterministic synthetic stream) are consecutive
    pieces of it; logparser_amd.shard.stream_split places the cuts at equal
    byte offsets (all_gather of the chunk sizes / line counts, all-reduce of
    the cuts, which also gives each split's global first line number).  The
    lines of this split outside the home chunk (next to a neighbour's) are
    produced the way a split reader reads past its end: from the stream
    itself (here, the deterministic generator) -- never moved between GPUs.
    Returns ((offset, bytes) of the split in buf, first lines, byte cuts)."""
    from logparser_amd.shard import stream_split
    home = buf[front:front + nbytes]
    first, pos = stream_split(nbytes, lines_per_rank,
                              lambda off, n: home[off:off + n].cpu().numpy(),
                              lambda a, b: device_terminators(torch, home[a:b]), device=device)
    h0, h1 = rank * lines_per_rank, (rank + 1) * lines_per_rank
    f0, f1 = first[rank], first[rank + 1]
    seed = SEEDS[workload]
    start, end = front, front + nbytes
    if f0 < h0:    # the split starts in the previous rank's chunk
        pre = lpa.synth(workload, seed, f0, h0 - f0)
        if len(pre) > front:
            raise RuntimeError("split prefix larger than the reserved front")
        buf[front - len(pre):front].copy_(torch.frombuffer(bytearray(pre), dtype=torch.uint8))
        start = front - len(pre)
    elif f0 > h0:
        start = front + len(lpa.synth(workload, seed, h0, min(f0, h1) - h0))
    if f1 > h1:    # the split ends in the next rank's chunk
        post = lpa.synth(workload, seed, h1, f1 - h1)
        if end + len(post) > buf.numel():
            raise RuntimeError("split suffix past the device buffer")
        buf[end:end + len(post)].copy_(torch.frombuffer(bytearray(post), dtype=torch.uint8))
        end += len(post)
    elif f1 < h1:
        end = front + nbytes - len(lpa.synth(workload, seed, max(f1, h0), h1 - max(f1, h0)))
    end = max(end, start)
    if buf.is_cuda:
        torch.cuda.synchronize()
    return (start, end - start), first, pos


def newline_batches(buf, off, nbytes, batch_bytes, probe=1 << 20):
    """[(offset, bytes)] pieces of buf[off, off + nbytes) of about batch_bytes
    each, every cut just after a '\n' (a line boundary whatever the
    terminators around it); one piece when batch_bytes is 0."""
    if not batch_bytes or nbytes <= batch_bytes:
        return [(off, nbytes)]
    out, a, end = [], off, off + nbytes
    while end - a > batch_bytes:
        c = a + batch_bytes
        w = bytes(buf[c:min(end, c + probe)].cpu().numpy())
        k = w.find(b"\n")
        if k < 0:
            break  # a line longer than the probe: the rest stays one piece
        out.append((a, c + k + 1 - a))
        a = c + k + 1
    if end > a:
        out.append((a, end - a))
    return out


def pcie_inclusive(torch, parser, buf, batches, max_bytes):
    """Host-resident batches (pinned), the rate a caller handing over host
    buffers sees (never the headline):
      serial     -- each batch copied H2D inside lp_parse_batch (BUF_HOST);
      overlapped -- double-buffered: the copy of batch i+1 into one aligned
                    device staging buffer (copy stream) runs while batch i is
                    parsed from the other (compute stream), one handle, so
                    the sticky routing state is carried as in the serial case."""
    n = 0
    sel = []
    for off, nb in batches:
        if n + nb > max_bytes and sel:
            break
        sel.append((off, nb))
        n += nb
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    hoff = []
    pos = 0
    for off, nb in sel:
        host[pos:pos + nb].copy_(buf[off:off + nb])
        hoff.append(pos)
        pos += nb
    torch.cuda.synchronize()
    lines = 0
    t0 = time.perf_counter()
    for (_, nb), h in zip(sel, hoff):
        lines += parser.run(host.data_ptr() + h, nb, on_device=False)["lines"]
    dt_serial = time.perf_counter() - t0

    big = max(nb for _, nb in sel)
    stage = [torch.empty(big + 4096, dtype=torch.uint8, device=buf.device) for _ in range(2)]
    cs, xs = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    lines2 = 0
    t0 = time.perf_counter()
    with torch.cuda.stream(xs):
        stage[0][:sel[0][1]].copy_(host[hoff[0]:hoff[0] + sel[0][1]], non_blocking=True)
    xs.synchronize()
    for i, (_, nb) in enumerate(sel):
        if i + 1 < len(sel):
            nb1, h1 = sel[i + 1][1], hoff[i + 1]
            with torch.cuda.stream(xs):
                stage[(i + 1) % 2][:nb1].copy_(host[h1:h1 + nb1], non_blocking=True)
        lines2 += parser.run(stage[i % 2].data_ptr(), nb, on_device=True, stream=cs.cuda_stream)["lines"]
        xs.synchronize()
    dt_over = time.perf_counter() - t0
    return {"value": round(n / dt_over / 1e9, 3), "unit": "GB/s", "lines_per_s": round(lines2 / dt_over, 1),
            "serial_value": round(n / dt_serial / 1e9, 3),
            "sample": "%d host-pinned batches (%.2f GB); value: double-buffered H2D (copy stream) overlapped with "
                      "index + parse (compute stream), one handle; serial_value: H2D copy inside each call" % (len(sel), n / 1e9),
            "lines": lines2}


def cpu_run(oracle_lib, lpa, workload, fields, sample_lines, threads, repeats, seconds):
    """Median of `repeats` timed oracle runs on `threads` threads over the
    first lines of the workload (about `seconds` of work per run)."""
    fmt = lpa.SYNTH_FORMATS[workload]
    probe = lpa.synth(workload, SEEDS[workload], 0, 2000)
    secs, _ = oracle_lib.bench(fmt, fields, probe, 1)
    rate1 = 2000 / max(secs, 1e-6)
    n = int(min(sample_lines, max(20000, rate1 * threads * seconds)))
    data = lpa.synth(workload, SEEDS[workload], 0, n)
    runs = []
    for _ in range(repeats):
        secs, counts = oracle_lib.bench(fmt, fields, data, threads)
        runs.append(secs)
    runs.sort()
    secs = runs[len(runs) // 2]
    return {"value": round(len(data) / secs / 1e9, 6), "lines_per_s": round(counts[0] / secs, 1), "cores": threads,
            "lines": counts[0], "bytes": len(data), "counts": counts, "seconds": round(secs, 2),
            "spread_gbs": [round(len(data) / t / 1e9, 6) for t in reversed(runs)]}


def usable_cpus():
    """CPUs this process may run on: its affinity mask, capped by a cgroup
    CPU quota (cgroup v2 cpu.max, v1 cpu.cfs_quota_us / cpu.cfs_period_us)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            q = float(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = float(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota:
        n = min(n, max(1, int(quota + 0.999)))
    return max(1, n)


def cpu_baseline(lpa, workload, fields, sample_lines, threads, repeats=3):
    """The oracle (C restatement of the reference semantics) on the GPU box's
    host cores, on the first lines of the same workload: a sweep of thread
    counts up to the CPUs this process may use (affinity and cgroup quota),
    one run each; the fastest count is run `repeats` times and its median is
    the value (every swept rate is reported, the value is at least each)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    oracle_lib.lib()
    usable = usable_cpus()
    if threads:
        counts = [threads]
    else:
        counts = sorted({c for c in (1, 4, usable // 2, usable, 2 * usable) if c >= 1})
    sweep = {}
    for t in counts:
        sweep[t] = cpu_run(oracle_lib, lpa, workload, fields, sample_lines, t, 1, 2)
    best_t = max(sweep, key=lambda t: sweep[t]["value"])
    full = cpu_run(oracle_lib, lpa, workload, fields, sample_lines, best_t, repeats, 3)
    if full["value"] < sweep[best_t]["value"]:  # the median of the repeats may fall below the sweep's single run
        full = dict(sweep[best_t], spread_gbs=full["spread_gbs"] + sweep[best_t]["spread_gbs"])
    c = full["counts"]
    return {
        "value": full["value"],
        "unit": "GB/s",
        "lines_per_s": full["lines_per_s"],
        "cores": min(best_t, usable),  # CPUs the run could occupy (threads beyond them time-share)
        "threads": best_t,
        "usable_cpus": usable,
        "host_cpus": os.cpu_count(),
        "kind": "port",
        "sample": "first %d lines (%.1f MB) of the config-%d workload, all %d paths, oracle/ C restatement, one parser "
                  "per thread; thread sweep %s over the %d CPUs this process may use (affinity / cgroup quota; the box "
                  "reports %d), the fastest (%d threads) as the median of %d runs; ok=%d bad=%d unsupported=%d" % (
                      full["lines"], full["bytes"] / 1e6, workload, len(fields), counts, usable, os.cpu_count(), best_t,
                      repeats, c[1], c[2], c[3]),
        "seconds": full["seconds"],
        "spread_gbs": full["spread_gbs"],
        "thread_sweep_gbs": {str(t): r["value"] for t, r in sorted(sweep.items())},
    }


# typed output columns of the delivery measurement (a Hive / ParsedRecord table)
TABLE_COLS = [("IP:connection.client.host", str), ("TIME.EPOCH:request.receive.time.epoch", int),
              ("HTTP.METHOD:request.firstline.method", str), ("HTTP.PATH:request.firstline.uri.path", str),
              ("STRING:request.status.last", str), ("BYTES:response.body.bytes", int),
              ("HTTP.HOST:request.referer.host", str), ("HTTP.USERAGENT:request.user-agent", str)]


def device_table(lpa, torch, parser, n_lines):
    """lp_result_table on the device view of the timed batch (every line, the
    TABLE_COLS present): values, offsets and bytes built in HBM; timed with
    the column buffers already sized (a first call reports the byte counts)."""
    r = lpa.BatchResult(parser)
    cols = [c for c in TABLE_COLS if c[0] in parser.fields]
    if not cols:
        return None
    t = r.table_device(cols)  # sizes the STRING columns' bytes
    caps = {p: int(v[0][1].numel()) + 16 for p, v in t.items() if dict(cols)[p] is str}
    del t
    # the output buffers allocated (and touched) before the timed call: the
    # timed region is lp_result_table alone (the three kernels and the scans)
    bufs = r.table_buffers(cols, chars_cap=caps)
    for b in bufs:
        for x in b:
            if x is not None:
                x.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t = r.table_device(cols, buffers=bufs)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ph = r.table_timing()
    nbytes = sum(int(v[0][1].numel()) if dict(cols)[p] is str else 0 for p, v in t.items())
    # k_table_chars: each STRING byte read once (input / arena) and written once
    chars_gbs = 2 * nbytes / (ph["chars"] / 1e3) / 1e9 if ph["chars"] > 0 else None
    del t, bufs
    n_lines = r.n_lines  # the handle's last batch
    return {"table_rows_per_s_device": round(n_lines / dt, 1), "table_seconds_device": round(dt, 4),
            "table_phase_ms": {k: round(v, 3) for k, v in ph.items()},
            "table_rows_per_s_kernels": round(n_lines / (sum(ph.values()) / 1e3), 1) if sum(ph.values()) > 0 else None,
            "table_chars_gbs": round(chars_gbs, 1) if chars_gbs else None,
            "table_chars_roofline_frac": round(chars_gbs / HBM_PEAK_GBS, 3) if chars_gbs else None,
            "table_columns": [c for c, _ in cols], "table_string_bytes": nbytes,
            "table_sample_device": "lp_result_table on the device view of the timed batch (%d lines, %d columns: "
                                   "values, Arrow offsets and bytes in HBM; output buffers allocated before the "
                                   "timed call; phases by HIP events)" % (n_lines, len(cols))}


def host_delivery(lpa, torch, parser, n_lines, workload, sample=100000):
    """Rate at which the finished batch reaches the caller: the typed columns
    built on the device (device_table); one lp_result_copy of the batch's SoA
    results (line index, columns, arena) into pinned host memory; then the
    host-side record rebuild (lp_result_record_json, one thread) and the host
    table from a copy of a small batch."""
    import ctypes
    L = lpa.lib()
    dtab = device_table(lpa, torch, parser, n_lines)
    need = -L.lp_result_copy(parser._h, None, 0, 0, None)
    host = torch.empty(need, dtype=torch.uint8, pin_memory=True)
    res = lpa.LpResult()
    t0 = time.perf_counter()
    rc = L.lp_result_copy(parser._h, ctypes.c_void_p(host.data_ptr()), need, 0, ctypes.byref(res))
    dt = time.perf_counter() - t0
    del host
    if rc < 0:
        return None
    data = lpa.synth(workload, SEEDS[workload], 0, sample)
    r = parser.parse_batch(data)
    _, res2 = r.copy_to_host()
    out = ctypes.create_string_buffer(1 << 16)
    ok = [i for i in range(r.n_lines) if r.status[i] == lpa.LINE_OK][:20000]
    t1 = time.perf_counter()
    for i in ok:
        L.lp_result_record_json(parser._h, ctypes.byref(res2), i, out, 1 << 16)
    dt2 = time.perf_counter() - t1
    # the same typed columns from the host copy (the replay), 16 host threads
    cols = [c for c in TABLE_COLS if c[0] in parser.fields]
    t2 = time.perf_counter()
    r.table_from(res2, cols, threads=16, decode=False)
    dt3 = time.perf_counter() - t2
    out = {"soa_copy_lines_per_s": round(n_lines / dt, 1), "soa_copy_gbs": round(need / dt / 1e9, 3),
           "soa_bytes": int(need), "records_json_per_s_1thread": round(len(ok) / dt2, 1),
           "table_rows_per_s_host_16threads": round(r.n_lines / dt3, 1),
           "sample": "lp_result_copy of the timed batch's SoA (%d lines) into pinned host memory; "
                     "lp_result_record_json of the %d OK lines of a %d-line batch, one host thread; "
                     "lp_result_table from a host copy of the same batch (the table columns, 16 threads)"
                     % (n_lines, len(ok), sample)}
    if dtab:
        out.update(dtab)
    return out


def pmc_traffic(path, n_lines, lib_path, kernel="k_parse_chunks"):
    """HBM bytes per launch of `kernel` measured by PMC counters, or None."""
    try:
        import hashlib
        d = json.load(open(path))
        sha = hashlib.sha256(open(lib_path, "rb").read()).hexdigest()
        if d.get("lines") != n_lines or d.get("lib_sha256") != sha:
            return None
        return d["kernels"][kernel]["hbm_bytes"]
    except (OSError, KeyError, ValueError):
        return None


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` started as one plain process (WORLD_SIZE unset):
    run N rank processes, one per GPU, through torch.distributed.run as a
    CHILD process (the parent has made no GPU call and never execs), and
    exit with its status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)
    log("bench: launching %d ranks: %s" % (n, " ".join(cmd)))
    return subprocess.call(cmd, env=dict(os.environ))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--lines", type=int, default=100_000_000, help="lines per GPU")
    ap.add_argument("--cpu-sample-lines", type=int, default=4_000_000)
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0 = sweep up to the usable CPUs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-delivery", action="store_true", help="skip the host delivery measurement (huge batches)")
    ap.add_argument("--workload", type=int, default=2, choices=(2, 3, 4, 5), help="BASELINE.json config")
    ap.add_argument("--batch-mb", type=int, default=None,
                    help="split the resident input into newline-aligned batches of about this size "
                         "(default: one batch; 1024 for --workload 5)")
    ap.add_argument("--fields", default="all",
                    help="all (the config-2 workload) | comma list of TYPE:path (profiling experiments only)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic_latest.json"),
                    help="tools/pmc_traffic.py summary of separate rocprofv3 --pmc passes; fills roofline.traffic "
                         "when it was taken on this workload with this exact engine build")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the first action, before torch or any GPU call: N rank processes
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d (one rank per GPU)" % (args.gpus, world))
    # rehearsal knobs (never used by the driver): LP_BENCH_DEVICE puts every
    # rank on one GPU, LP_BENCH_BACKEND=gloo replaces RCCL, so the N-rank
    # path can run on a one-GPU box; LP_BENCH_DRYRUN stops every rank right
    # after the process group is up, before any GPU call (CPU tests of the
    # launcher)
    dry = bool(os.environ.get("LP_BENCH_DRYRUN"))
    backend = None
    if world > 1:
        backend = "gloo" if dry else os.environ.get("LP_BENCH_BACKEND", "nccl")
    if dry:
        if world > 1:
            dist.init_process_group(backend)
            world = dist.get_world_size()
            dist.barrier()
            dist.destroy_process_group()
        print(json.dumps({"dryrun": True, "rank": rank, "world_size": world, "gpus": args.gpus,
                          "backend": backend}), flush=True)
        return

    import logparser_amd as lpa
    from logparser_amd.shard import max_over_ranks, reduce_counters

    if os.environ.get("LP_BENCH_DEVICE"):
        local = int(os.environ["LP_BENCH_DEVICE"])
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()
        if world != args.gpus:
            raise SystemExit("bench: process group has %d ranks, --gpus %d" % (world, args.gpus))

    wl = args.workload
    fmt = lpa.SYNTH_FORMATS[wl]
    fields = lpa.get_possible_paths(fmt) if args.fields == "all" else args.fields.split(",")
    log("rank %d/%d: generating %d lines (config %d, seed %d) on %s" % (rank, world, args.lines, wl, SEEDS[wl], device))
    batch_mb = args.batch_mb if args.batch_mb is not None else (1024 if wl == 5 else 0)
    front = (256 << 20) if world > 1 else 0
    buf, nbytes, batches = generate_to_device(lpa, torch, wl, rank * args.lines, args.lines, device,
                                              batch_bytes=0 if world > 1 else batch_mb << 20, front=front)
    split = None
    if world > 1:
        # one stream, newline-aligned Hadoop splits.  Config 5 too: its
        # LogFormats are mutually exclusive, so the sticky
        # format state a split starts with changes no line's result
        # (tests/test_multirank.py checks this against the oracle)
        (soff, sbytes), first, cuts = split_stream(lpa, torch, buf, front, nbytes, wl, args.lines, rank, device)
        batches = newline_batches(buf, soff, sbytes, batch_mb << 20)
        nbytes = sbytes
        split = {"first_line": first, "byte_cuts": cuts}
        log("rank %d split: lines [%d, %d), bytes [%d, %d)" % (rank, first[rank], first[rank + 1], cuts[rank],
                                                                cuts[rank + 1]))
    log("input resident in HBM: %.2f GB in %d batch(es)" % (nbytes / 1e9, len(batches)))

    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(device)[0]
    parser = lpa.HttpdLoglineParser(fmt, fields, device=local)
    counters = torch.zeros(4, dtype=torch.int64, device=device)

    def step():
        st = None
        for off, nb in batches:
            r = parser.run(buf.data_ptr() + off, nb, on_device=True)
            if st is None:
                st = r
            else:
                for k in ("lines", "ok", "bad", "fallback", "ms_total", "ms_index", "ms_parse", "bytes_in", "bytes_out",
                          "overflow_waves", "retries", "ms_parse_kernels", "ms_uri_kernels", "bytes_parse_kernels",
                          "bytes_uri_kernels"):
                    st[k] += r[k]
        if world > 1:
            counters.copy_(torch.tensor([st["lines"], st["ok"], st["bad"], st["fallback"]], dtype=torch.int64))
            reduce_counters(counters)  # RCCL all-reduce: the only cross-GPU traffic
        return st

    for _ in range(args.warmup):
        st = step()
    torch.cuda.synchronize()
    engine_hbm = free0 - torch.cuda.mem_get_info(device)[0]  # the handle's buffers after the warmup batches
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    parse_ms, index_ms, pk_ms, uk_ms, stats = [], [], [], [], None
    for _ in range(args.steps):
        stats = step()
        parse_ms.append(stats["ms_parse"])
        index_ms.append(stats["ms_index"])
        pk_ms.append(stats["ms_parse_kernels"])
        uk_ms.append(stats["ms_uri_kernels"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, device=device)

    if split is not None:  # the whole stream, every split once per step
        total_bytes = split["byte_cuts"][-1] * args.steps
        total_lines = split["first_line"][-1] * args.steps
        if int(counters[0]) != split["first_line"][-1]:
            raise RuntimeError("all-reduced line count %d != the stream's %d" % (int(counters[0]), split["first_line"][-1]))
    else:
        total_bytes = nbytes * world * args.steps
        total_lines = stats["lines"] * world * args.steps
    avg_parse = sum(parse_ms) / len(parse_ms)
    avg_pk, avg_uk = sum(pk_ms) / len(pk_ms), sum(uk_ms) / len(uk_ms)
    algo_bytes = stats["bytes_in"] + stats["bytes_out"]
    pass_gbs = algo_bytes / (avg_parse / 1e3) / 1e9
    # the dominant kernel: k_parse_chunks (the parse kernels' HIP-event time on
    # the launch stream; their algorithmic bytes: the input once, the line
    # index, their columns)
    pk_bytes, uk_bytes = stats["bytes_parse_kernels"], stats["bytes_uri_kernels"]
    achieved = pk_bytes / (avg_pk / 1e3) / 1e9
    uri_gbs = uk_bytes / (avg_uk / 1e3) / 1e9 if avg_uk > 0 else 0.0
    with_pmc = wl == 2 and args.fields == "all"
    # the dominant kernel: the one-pass chunked parse (several LogFormats: its
    # routing instance, k_parse_chunks<.., MF>, since round 6)
    pk_name = "k_parse_chunks" if len(fmt.split("\n")) == 1 else "k_parse_chunks (several LogFormats: routing instance)"

    result = {
        "metric": "GB/s (and lines/s) of 'combined' log parsed per GPU and per 8xMI355X node",
        "value": round(total_bytes / elapsed / 1e9, 3),
        "unit": "GB/s",
        "lines_per_s": round(total_lines / elapsed, 1),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (lp_synth workload %d, seed %d; deterministic per line)" % (wl, SEEDS[wl]),
        "config": {
            "workload": (WORKLOAD_NAMES[wl] % stats["lines"]) + " per GPU (%.2f GB), all %d paths requested "
                        "(epoch, first line, URI parts, query params), input resident in HBM" % (nbytes / 1e9, len(fields)),
            "logformat": fmt,
            "lines_per_gpu": stats["lines"],
            "bytes_per_gpu": nbytes,
            "mean_line_bytes": round(nbytes / max(1, stats["lines"]), 1),
            "mean_line_note": "incl. the terminator; the config-2 generator draws every field of SURVEY.md 8(d) "
                              "(request URIs and referers with query strings, full user-agent strings), which "
                              "makes its lines longer than the reference demo log's 230.5 B: lines_per_s is the "
                              "length-independent figure" if wl == 2 else "incl. the terminator",
            "parallelism": ("dp%d (one stream in Hadoop newline-aligned splits: all_gather of chunk sizes, "
                            "all-reduce of the cuts; %s counter all-reduce per step)"
                            % (world, "RCCL" if backend == "nccl" else backend)) if split is not None else
                           "dp1 (one rank: no collective)",
            "world_size": world,
            "backend": backend,
            "batches_per_step": len(batches),
        },
        # this rank's (rank 0's) batch; with several ranks the all-reduced
        # totals are status_counts_all_ranks
        "status_counts": {k: int(stats[k]) for k in ("lines", "ok", "bad", "fallback")},
        "parse_diag": {"overflow_waves": int(stats.get("overflow_waves", 0)), "retries": int(stats.get("retries", 0)),
                       "waves": (int(stats["lines"]) + 63) // 64},
        "hbm_footprint": {"input_bytes": int(nbytes), "engine_bytes": int(engine_hbm),
                          "engine_bytes_per_line": round(engine_hbm / max(1, stats["lines"]), 1),
                          "note": "device memory the handle holds after the warmup (columns, line index, arena, "
                                  "scratch), measured with hipMemGetInfo; the input is the caller's"},
        "kernel_ms": {"parse_avg": round(avg_parse, 3), "index_avg": round(sum(index_ms) / len(index_ms), 3),
                      "parse_kernels_avg": round(avg_pk, 3), "uri_kernels_avg": round(avg_uk, 3)},
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic(args.pmc_json, stats["lines"], lpa.LIB_PATH, pk_name) if with_pmc else None,
            "kernel": pk_name,
            "ms_per_launch": round(avg_pk, 3),
            "algorithmic_bytes_per_launch": int(pk_bytes),
            "bytes_per_line": round(pk_bytes / max(1, stats["lines"]), 1),
            "uri_kernel": {
                "kernel": "k_uri_lines", "ms_per_launch": round(avg_uk, 3), "achieved": round(uri_gbs, 1),
                "frac": round(uri_gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": int(uk_bytes),
                "bytes_per_line": round(uk_bytes / max(1, stats["lines"]), 1),
                "traffic": pmc_traffic(args.pmc_json, stats["lines"], lpa.LIB_PATH, "k_uri_lines") if with_pmc else None,
            },
            "parse_pass": {
                "kernels": "k_parse_chunks (+ k_parse_deferred, k_route_ovf, k_parse_ovf_lines) + k_uri_lines (+ its overflow path, counter reduction)",
                "ms": round(avg_parse, 3), "achieved": round(pass_gbs, 1), "frac": round(pass_gbs / HBM_PEAK_GBS, 4),
                "algorithmic_bytes": int(algo_bytes), "bytes_per_line": round(algo_bytes / max(1, stats["lines"]), 1),
            },
        },
        "cpu_baseline": None,
    }
    # run histograms of the last step's batch (device kernel), all-reduced over the ranks
    # (outside the timed region)
    hist = torch.zeros(lpa.HIST_WORDS, dtype=torch.int64, device=device)
    if len(batches) == 1:
        parser.histograms(device_ptr=hist.data_ptr())
        reduce_counters(hist)
        hd = lpa.decode_histograms(hist.cpu().tolist())
        top = sorted(hd["status"].items(), key=lambda kv: -kv[1])[:6]
        result["histograms"] = {"lines": hd["lines"], "ok": hd["ok"], "bad": hd["bad"], "fallback": hd["fallback"],
                                "status_top": {str(c): v for c, v in top}, "methods": hd["methods"],
                                "note": "lp_histograms of the last step (all ranks, RCCL all-reduce), untimed"}
    if wl == 5:
        result["config"]["formats"] = fmt.split("\n")
        result["config"]["corpus_bytes_all_ranks"] = total_bytes
        if rank == 0:
            result["pcie_inclusive"] = pcie_inclusive(torch, parser, buf, batches, 8 << 30)
    if world > 1:
        result["status_counts_all_ranks"] = {k: int(counters[j]) for j, k in enumerate(("lines", "ok", "bad", "fallback"))}
    if rank == 0 and wl != 5 and not args.no_delivery:
        result["delivery"] = host_delivery(lpa, torch, parser, stats["lines"], wl)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline (oracle, %s threads) ..." % (args.cpu_threads or "sweep of"))
        result["cpu_baseline"] = cpu_baseline(lpa, wl, fields, args.cpu_sample_lines, args.cpu_threads)
        # vs_baseline stays null: BASELINE.md publishes no number for this metric
        result["vs_cpu_baseline"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
