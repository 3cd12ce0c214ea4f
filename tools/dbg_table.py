"""Debug helper: device vs host table of one column on the remap corpus."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np
import logparser_amd as lpa
import remap_corpus as rc

lines = rc.corpus(3, 3000)
p = lpa.HttpdLoglineParser(rc.FORMAT, rc.FIELDS)
for n, t in rc.REMAPS:
    p.add_type_remapping(n, t)
r = p.parse_batch(b"".join(l + b"\n" for l in lines))
_, res = r.copy_to_host()
for path in sys.argv[1:]:
    col = [(path, str)]
    h = r.table_from(res, col, decode=True)[path]
    d = r.table_device(col)[path]
    (off, chars), ok = d
    off = off.cpu().numpy(); chars = chars.cpu().numpy().tobytes(); ok = ok.cpu().numpy()
    bad = 0
    for i in range(r.n_lines):
        dv = chars[off[i]:off[i + 1]].decode() if ok[i] else None
        if dv != h[0][i]:
            bad += 1
            if bad < 5:
                print(path, i, "status", r.status[i], "host", repr(h[0][i]), "device", repr(dv))
                print("   rec:", {k: v for k, v in r.record(i).items() if "next" in k} if r.status[i] == 0 else None)
    print(path, "mismatches", bad)
