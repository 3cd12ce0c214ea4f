"""Print per-kernel SQ counter values from tools/sq_counters.sh output."""
import csv
import glob
import re
import sys

d = sys.argv[1]
vals = {}
for f in sorted(glob.glob(d + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        m = re.search(r"::(k_\w+)(?:<[^>]*>)?\(", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:40]
        vals.setdefault(k, {})[r["Counter_Name"]] = float(r["Counter_Value"])
for k, v in vals.items():
    if not (k.startswith("k_parse") or k.startswith("k_uri")):
        continue
    print(k)
    for c in sorted(v):
        print("  %-24s %16.0f" % (c, v[c]))
    w = v.get("SQ_WAVES", 0)
    if w:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_FLAT",
                  "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in v:
                print("  per wave %-16s %10.0f" % (c, v[c] / w))
