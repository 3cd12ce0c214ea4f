"""Parse-kernel time of synthetic config-N lines for several LP_OPT_CHUNK_LINES
values (lines per byte chunk of k_parse_chunks): the chunk size trades LDS per
wave (waves per CU) against lanes per wave.  Usage: chunk_sweep.py LINES
[counts, comma separated]."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import logparser_amd as lpa  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
counts = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,32,40,48,56,64").split(",")]
wl = int(os.environ.get("LP_WORKLOAD", "2"))
fmt = lpa.SYNTH_FORMATS[wl]
fields = lpa.get_possible_paths(fmt)
data = lpa.synth(wl, 20261015, 0, n)
t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
for cl in counts:
    p = lpa.HttpdLoglineParser(fmt, fields, options={lpa.OPT_CHUNK_LINES: cl} if cl else None)
    for _ in range(2):
        p.run(t.data_ptr(), len(data))
    ks, us = [], []
    for _ in range(5):
        st = p.run(t.data_ptr(), len(data))
        ks.append(st["ms_parse_kernels"])
        us.append(st["ms_uri_kernels"])
    print("chunk_lines %2d  parse kernels %.3f ms  uri kernels %.3f ms  ok %d fallback %d ovf %d" %
          (cl, min(ks), min(us), st["ok"], st["fallback"], st["overflow_waves"]), flush=True)
