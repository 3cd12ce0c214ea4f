"""Device-table phases on N synthetic config-2 lines (the bench's TABLE_COLS):
lp_result_table on the device view, buffers allocated before the timed
calls; prints the HIP-event phase times.  Usage: table_bench.py [LINES]."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import logparser_amd as lpa  # noqa: E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
fields = lpa.get_possible_paths("combined")
data = lpa.synth(2, 20261015, 0, n)
t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
p = lpa.HttpdLoglineParser("combined", fields)
p.run(t.data_ptr(), len(data))
r = lpa.BatchResult(p)
cols = [c for c in bench.TABLE_COLS if c[0] in fields]
first = r.table_device(cols)
caps = {k: int(v[0][1].numel()) + 16 for k, v in first.items() if dict(cols)[k] is str}
del first
bufs = r.table_buffers(cols, chars_cap=caps)
for _ in range(3):
    r.table_device(cols, buffers=bufs)
    torch.cuda.synchronize()
    print(r.table_timing(), flush=True)
