"""Debug helper: the golden-vector groups on the GPU one by one, printing
each group before it runs (locates a crash) and the raw columns of its
first OK line."""
import faulthandler
import os
import sys
faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401
import golden_check
import logparser_amd as lpa
vec = golden_check.load_vectors()
groups = {}
for c in vec["cases"]:
    groups.setdefault((c["logformat"], tuple(c["fields"])), []).append(c)
for gi, ((fmt, fields), cases) in enumerate(groups.items()):
    print("group", gi, repr(fmt)[:80], len(fields), "fields", len(cases), "lines", flush=True)
    p = lpa.HttpdLoglineParser(fmt, list(fields))
    data = b"".join(c["line"].encode() + b"\n" for c in cases)
    r = p.parse_batch(data)
    buf, res = r.copy_to_host()
    cols = r.columns(res)
    for i in range(r.n_lines):
        if r.status[i] != lpa.LINE_OK:
            continue
        info = {k: int(v[i]) for k, v in cols.items() if k[0] in ("arena_base", "u_flags", "q_count", "q_params")}
        print("  line", i, info, flush=True)
        print("  ", r.record_json_from(res, i)[:120], flush=True)
