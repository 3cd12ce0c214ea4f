"""Run the LP_PROFILE build on synthetic config-2 lines and print cycles per
wave between the instrumentation points of k_parse_lines."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LOGPARSER_AMD_LIB"] = os.path.join(ROOT, "logparser_amd", "_dbg", "liblogparser_amd_prof.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
import logparser_amd as lpa  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
fields = lpa.get_possible_paths("combined") if len(sys.argv) < 3 else sys.argv[2].split(",")
data = lpa.synth_combined(20261015, 0, n)
t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
p = lpa.HttpdLoglineParser("combined", fields)
L = lpa.lib()
L.lp_profile_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
L.lp_profile_read_elems.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 128)()
el = (ctypes.c_ulonglong * 128)()
p.run(t.data_ptr(), len(data))
L.lp_profile_read(buf, 64)  # clear after warm-up
L.lp_profile_read_elems(el, 64)
st = p.run(t.data_ptr(), len(data))
L.lp_profile_read(buf, 64)
L.lp_profile_read_elems(el, 64)
names = {0: "start", 1: "staged", 2: "phase1 entry", 3: "guard", 4: "match", 5: "tok flags", 6: "time",
         7: "first line", 8: "arena need", 9: "phase1 exit", 10: "uri0 in", 11: "uri0 out", 12: "uri1 in",
         13: "uri1 out", 20: "phase2 exit", 21: "rows written", 22: "query pieces"}
for u in range(2):
    for j, nm in enumerate(["pass1", "authority", "path", "query", "frag"]):
        names[30 + 8 * u + j] = "u%d %s done" % (u, nm)
for u in range(2):
    names[50 + 4 * u] = "u%d walk start" % u
    names[51 + 4 * u] = "u%d fast walk" % u
    names[52 + 4 * u] = "u%d gen walk" % u
order = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 50, 51, 52, 30, 31, 32, 33, 34, 11, 12, 54, 55, 56, 38, 39, 40, 41, 42, 13,
         20, 21, 22]
pts = [k for k in order if buf[2 * k + 1]]
print("parse ms %.3f  waves %d" % (st["ms_parse"], buf[1]))
prev = None
for k in pts:
    s, c = buf[2 * k], buf[2 * k + 1]
    if prev is not None:
        ps, pc = buf[2 * prev], buf[2 * prev + 1]
        if c == pc:
            print("  %-14s -> %-14s %10.0f cycles/wave" % (names[prev], names[k], (s - ps) / c))
        else:
            print("  %-14s -> %-14s (mark counts differ %d vs %d)" % (names[prev], names[k], pc, c))
    prev = k
print("first-leaf elements (cycles per visit):")
print(p.describe())
for i in range(64):
    if el[2 * i + 1]:
        print("  elem %2d %10.0f" % (i, el[2 * i] / el[2 * i + 1]))
