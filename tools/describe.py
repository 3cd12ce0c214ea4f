"""Print the device program (lp_describe) of a BASELINE.json workload's LogFormat."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import logparser_amd as lpa
wl = int(sys.argv[1]) if len(sys.argv) > 1 else 2
fmt = lpa.SYNTH_FORMATS[wl]
p = lpa.HttpdLoglineParser(fmt, lpa.get_possible_paths(fmt))
p.parse_batch(lpa.synth(wl, 1, 0, 1000))
print(p.describe())
