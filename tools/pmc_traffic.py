"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) into
HBM bytes per launch of each kernel, with the gfx950 correction of
MI355X_MICROARCH.md (FETCH_SIZE reports 1/2 of the bytes of wide streaming
reads: doubled here; both counters are in KiB).

Only the bench batch's launches count: a kernel's dispatches shorter than
half its longest one (e.g. the small batch bench.py's delivery measurement
parses through the same handle, at the same grid size) are left out, and
the dispatch ids used are recorded.

  python tools/pmc_traffic.py <fetch counter csv> <write counter csv> [--lines N] [--out pmc.json]
"""
import argparse
import csv
import hashlib
import re
import json
from collections import defaultdict


def per_kernel(path, counter):
    rows = defaultdict(list)  # kernel -> [(duration ns, dispatch id, bytes)]
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        m = re.search(r"::(k_\w+)(?:<[^>]*>)?\(", name)
        short = m.group(1) if m else name[:60]
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        rows[short].append((dur, int(r["Dispatch_Id"]), float(r["Counter_Value"]) * 1024.0))
    out = {}
    for k, v in rows.items():
        longest = max(d for d, _, _ in v)
        keep = [(i, b) for d, i, b in v if d >= longest / 2]
        out[k] = (sum(b for _, b in keep) / len(keep), [i for i, _ in keep], len(v))
    return out


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
    out = {"note": "bytes per launch (mean over the dispatches at least half as long as the kernel's longest, i.e. "
                   "the bench batch's); fetch = FETCH_SIZE x 1024 x 2 (gfx950 correction), write = WRITE_SIZE x 1024",
           "lines": a.lines, "lib_sha256": lib_sha(a.lib) if a.lib else None, "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fb, fi, fn = f.get(k, (0.0, [], 0))
        wb, wi, wn = w.get(k, (0.0, [], 0))
        out["kernels"][k] = {"fetch_bytes": fb * 2.0, "write_bytes": wb, "hbm_bytes": fb * 2.0 + wb,
                             "fetch_dispatches": fi, "write_dispatches": wi, "dispatches_seen": [fn, wn]}
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
