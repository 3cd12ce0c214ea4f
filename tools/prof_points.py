"""Run the LP_PROFILE build on synthetic config-2 lines and print the mean
cycles per wave between consecutive instrumentation points of the parse kernel
(k_parse_chunks, or k_parse_lines for several LogFormats) and k_uri_lines
(per-wave timestamps, no atomics)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LOGPARSER_AMD_LIB"] = os.environ.get("LP_PROF_LIB") or os.path.join(ROOT, "logparser_amd", "_dbg", "liblogparser_amd_prof.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
import logparser_amd as lpa  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
wl = int(os.environ.get("LP_WORKLOAD", "2"))  # BASELINE.json config (lp_synth workload)
fmt = lpa.SYNTH_FORMATS[wl]
fields = lpa.get_possible_paths(fmt) if len(sys.argv) < 3 else sys.argv[2].split(",")
data = lpa.synth(wl, 20261015, 0, n)
t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
p = lpa.HttpdLoglineParser(fmt, fields)
L = lpa.lib()
W, K = 16384, 96
L.lp_profile_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(W * K, dtype=np.uint64)
p.run(t.data_ptr(), len(data))
p.run(t.data_ptr(), len(data))
L.lp_profile_read(buf.ctypes.data, W * K)  # clear after warm-up
st = p.run(t.data_ptr(), len(data))
L.lp_profile_read(buf.ctypes.data, W * K)
T = buf.reshape(W, K).astype(np.int64)
names = {0: "start", 1: "staged", 2: "phase1 entry", 3: "guard", 4: "match", 5: "tok flags", 6: "time",
         7: "first line", 9: "phase1 exit", 10: "uri0 in", 11: "uri0 out", 12: "uri1 in",
         13: "uri1 out", 21: "phase2 exit", 22: "query pieces", 23: "uri kernel start", 24: "uri copied",
         25: "uri plane", 26: "uri arena", 43: "scheme", 44: "auth end", 45: "ipv4", 46: "hostname", 47: "port",
         60: "chunk staged", 61: "line numbers", 62: "rows written",
         14: "strf parsed", 15: "strf resolved", 16: "strf fields", 27: "uri lane", 28: "uri gather loads",
         17: "q slots loaded", 18: "q prepared", 19: "q spill allocated"}
for u in range(2):
    for j, nm in enumerate(["pass1", "authority", "path", "query", "frag"]):
        names[30 + 8 * u + j] = "u%d %s done" % (u, nm)
for u in range(2):
    names[50 + 4 * u] = "u%d walk start" % u
    names[51 + 4 * u] = "u%d fast walk" % u
    names[52 + 4 * u] = "u%d gen walk" % u
# the parse kernel, then the URI kernel (k_uri_lines): separate orders
orders = [[0, 60, 1, 2, 3, 4, 5, 14, 15, 16, 6, 7, 9, 61, 62],
          [23, 27, 28, 24, 25, 26, 10, 50, 51, 52, 30, 31, 32, 33, 34, 11, 12, 54, 55, 56, 38, 43, 44, 45, 46, 47, 39, 40, 41, 42, 13, 21, 17, 18, 19, 22]]
print("parse ms %.3f  waves profiled %d" % (st["ms_parse"], int((T[:, 0] != 0).sum())))
for order in orders:
    acc = {}
    for w in range(W):
        row = T[w]
        prev = None
        for k in order:
            if row[k] == 0:
                continue
            if prev is not None:
                d = acc.setdefault((prev, k), [0.0, 0])
                d[0] += row[k] - row[prev]
                d[1] += 1
            prev = k
    for (a, b), (s_, c) in sorted(acc.items(), key=lambda kv: order.index(kv[0][0]) * 100 + order.index(kv[0][1])):
        print("  %-18s -> %-18s %9.0f cycles/wave  (%d waves)" % (names[a], names[b], s_ / c, c))
    rows = [r for r in T if r[order[0]] and r[order[-1]]]
    if rows:
        print("  kernel total %.0f cycles per wave" % np.mean([r[order[-1]] - r[order[0]] for r in rows]))

# first-leaf match cycles per element (LP_PROF_EL, slots 64 + i), k_parse_lines waves
el = T[:, 64:96]
rows = T[:, 0] != 0
if rows.any():
    m = el[rows].mean(axis=0)
    print("first-leaf element cycles per wave:", " ".join("%d:%.0f" % (i, v) for i, v in enumerate(m) if v))
print(p.describe())
