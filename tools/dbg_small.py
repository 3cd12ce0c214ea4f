"""Debug helper: one small config-2 batch through the engine, with
faulthandler, printing counters (run on the GPU box)."""
import faulthandler
import sys
import os
faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401
import logparser_amd as lpa
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
fields = lpa.get_possible_paths("combined") if len(sys.argv) < 3 else sys.argv[2].split(",")
data = lpa.synth_combined(20261015, 0, n)
p = lpa.HttpdLoglineParser("combined", fields)
print("compiled", flush=True)
r = p.parse_batch(data)
print("parsed", r.counters, r.diag, flush=True)
print(r.record_json(0)[:300], flush=True)
