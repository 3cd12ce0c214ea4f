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

  python bench.py [--gpus N] [--steps K] [--warmup W] [--lines L] [--workload 2|3|4]
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
SEEDS = {2: 20261015, 3: 20261016, 4: 20261017}
WORKLOAD_NAMES = {2: "config 2: %d synthetic 'combined' lines",
                  3: "config 3: %d synthetic 'combinedio' + %%{%%d/%%b/%%Y %%T}t.%%{msec_frac}t lines (5%% malformed)",
                  4: "config 4: %d synthetic NGINX '$request_time $upstream_response_time $pipe' lines"}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def generate_to_device(lpa, torch, workload, first_line, n_lines, device, chunk=1 << 20, workers=16):
    """Deterministic synthetic lines [first_line, first_line+n_lines) straight
    into one HBM buffer (host generation in parallel chunks, H2D in order)."""
    upper = n_lines * 320 + (1 << 20)
    dev = torch.empty(upper, dtype=torch.uint8, device=device)
    pos = 0
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
            if pos + len(data) > upper:
                raise RuntimeError("synthetic data larger than the device buffer bound")
            host = torch.frombuffer(bytearray(data), dtype=torch.uint8)
            dev[pos:pos + len(data)].copy_(host)
            pos += len(data)
            done += 1
            if done % 16 == 0:
                log("  generated %d/%d chunks (%.1f GB, %.0f s)" % (done, len(starts), pos / 1e9, time.time() - t0))
    torch.cuda.synchronize()
    return dev, pos


def cpu_baseline(lpa, workload, fields, sample_lines, threads):
    """The oracle (C restatement of the reference semantics) on the GPU box's
    host cores, on the first sample_lines lines of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    oracle_lib.lib()
    fmt = lpa.SYNTH_FORMATS[workload]
    probe = lpa.synth(workload, SEEDS[workload], 0, 2000)
    secs, _ = oracle_lib.bench(fmt, fields, probe, 1)
    rate1 = 2000 / max(secs, 1e-6)
    # aim at ~15 s of work on `threads` threads
    n = int(min(sample_lines, max(20000, rate1 * threads * 15)))
    data = lpa.synth(workload, SEEDS[workload], 0, n)
    secs, counts = oracle_lib.bench(fmt, fields, data, threads)
    return {
        "value": round(len(data) / secs / 1e9, 6),
        "unit": "GB/s",
        "lines_per_s": round(counts[0] / secs, 1),
        "cores": threads,
        "kind": "port",
        "sample": "first %d lines (%.1f MB) of the config-%d workload, all %d paths, oracle/ C restatement, "
                  "%d threads, one parser per thread; ok=%d bad=%d unsupported=%d" % (
                      counts[0], len(data) / 1e6, workload, len(fields), threads, counts[1], counts[2], counts[3]),
        "seconds": round(secs, 2),
    }


def pmc_traffic(path, n_lines, lib_path):
    """HBM bytes per k_parse_lines launch measured by PMC counters, or None."""
    try:
        import hashlib
        d = json.load(open(path))
        sha = hashlib.sha256(open(lib_path, "rb").read()).hexdigest()
        if d.get("lines") != n_lines or d.get("lib_sha256") != sha:
            return None
        return d["kernels"]["k_parse_lines"]["hbm_bytes"]
    except (OSError, KeyError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--lines", type=int, default=100_000_000, help="lines per GPU")
    ap.add_argument("--cpu-sample-lines", type=int, default=2_000_000)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", type=int, default=2, choices=(2, 3, 4), help="BASELINE.json config")
    ap.add_argument("--fields", default="all",
                    help="all (the config-2 workload) | comma list of TYPE:path (profiling experiments only)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic_latest.json"),
                    help="tools/pmc_traffic.py summary of separate rocprofv3 --pmc passes; fills roofline.traffic "
                         "when it was taken on this workload with this exact engine build")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import logparser_amd as lpa
    from logparser_amd.shard import max_over_ranks, reduce_counters

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    wl = args.workload
    fmt = lpa.SYNTH_FORMATS[wl]
    fields = lpa.get_possible_paths(fmt) if args.fields == "all" else args.fields.split(",")
    log("rank %d/%d: generating %d lines (config %d, seed %d) on %s" % (rank, world, args.lines, wl, SEEDS[wl], device))
    buf, nbytes = generate_to_device(lpa, torch, wl, rank * args.lines, args.lines, device)
    log("input resident in HBM: %.2f GB" % (nbytes / 1e9))

    parser = lpa.HttpdLoglineParser(fmt, fields, device=local)
    counters = torch.zeros(4, dtype=torch.int64, device=device)

    def step():
        st = parser.run(buf.data_ptr(), nbytes, on_device=True)
        if world > 1:
            counters.copy_(torch.tensor([st["lines"], st["ok"], st["bad"], st["fallback"]], dtype=torch.int64))
            reduce_counters(counters)  # RCCL all-reduce: the only cross-GPU traffic
        return st

    for _ in range(args.warmup):
        st = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    parse_ms, index_ms, stats = [], [], None
    for _ in range(args.steps):
        stats = step()
        parse_ms.append(stats["ms_parse"])
        index_ms.append(stats["ms_index"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, device=device)

    total_bytes = nbytes * world * args.steps
    total_lines = stats["lines"] * world * args.steps
    avg_parse = sum(parse_ms) / len(parse_ms)
    algo_bytes = stats["bytes_in"] + stats["bytes_out"]
    achieved = algo_bytes / (avg_parse / 1e3) / 1e9

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
            "parallelism": "dp%d (newline-aligned shards, RCCL counter all-reduce)" % world,
        },
        "status_counts": {k: int(stats[k]) for k in ("lines", "ok", "bad", "fallback")},
        "kernel_ms": {"parse_avg": round(avg_parse, 3), "index_avg": round(sum(index_ms) / len(index_ms), 3)},
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic(args.pmc_json, stats["lines"], lpa.LIB_PATH) if wl == 2 and args.fields == "all" else None,
            "kernel": "k_parse_lines",
            "algorithmic_bytes_per_launch": int(algo_bytes),
            "bytes_per_line": round(algo_bytes / max(1, stats["lines"]), 1),
        },
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline (oracle, %d threads) ..." % args.cpu_threads)
        result["cpu_baseline"] = cpu_baseline(lpa, wl, fields, args.cpu_sample_lines, args.cpu_threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
