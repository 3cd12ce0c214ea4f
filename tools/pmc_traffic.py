"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) into
HBM bytes per launch of each kernel, with the gfx950 correction of
MI355X_MICROARCH.md (FETCH_SIZE reports 1/2 of the bytes of wide streaming
reads: doubled here; both counters are in KiB).

  python tools/pmc_traffic.py <fetch counter csv> <write counter csv> [--lines N] [--out pmc.json]
"""
import argparse
import csv
import hashlib
import re
import json
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        m = re.search(r"::(k_\w+)(?:<\w+>)?\(", name)
        short = m.group(1) if m else name[:60]
        acc[short].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def lib_sha(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--lines", type=int, default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--lib", default=None, help="engine .so the counters were taken with (its sha256 is recorded)")
    a = ap.parse_args()
    f = per_kernel(a.fetch, "FETCH_SIZE")
    w = per_kernel(a.write, "WRITE_SIZE")
    out = {"note": "bytes per launch; fetch = FETCH_SIZE x 1024 x 2 (gfx950 correction), write = WRITE_SIZE x 1024",
           "lines": a.lines, "lib_sha256": lib_sha(a.lib) if a.lib else None, "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fb = f.get(k, 0.0) * 2.0
        wb = w.get(k, 0.0)
        out["kernels"][k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb}
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
