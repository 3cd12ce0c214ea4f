"""GPU debugging aid: parse one golden group as a batch and line by line,
print device records next to the emulation's."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import emu_lib  # noqa: E402
import logparser_amd as lpa  # noqa: E402

v = json.load(open(os.path.join(ROOT, "tests/golden/reference_vectors.json")))
src = sys.argv[1] if len(sys.argv) > 1 else "hpt/ApacheHttpdLogParserTest.java:365-370"
case = [c for c in v["cases"] if c["source"] == src][0]
group = [c for c in v["cases"] if c["logformat"] == case["logformat"] and c["fields"] == case["fields"]]
p = lpa.HttpdLoglineParser(case["logformat"], case["fields"])
e = emu_lib.Emu(case["logformat"], case["fields"])
data = b"".join(c["line"].encode() + b"\n" for c in group)
r = p.parse_batch(data)
for i, c in enumerate(group):
    print("LINE", i, repr(c["line"]), "status", r.status[i], flush=True)
    if r.status[i] == 0:
        print("  gpu  ", r.record_json(i), flush=True)
    print("  emu  ", e.parse_raw(c["line"]), flush=True)
p2 = lpa.HttpdLoglineParser(case["logformat"], case["fields"])
for i, c in enumerate(group):
    r1 = p2.parse_batch(c["line"].encode() + b"\n")
    print("  alone", i, r1.record_json(0) if r1.status[0] == 0 else r1.status[0], flush=True)
