import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import logparser_amd as lpa, oracle_lib
fields = oracle_lib.possible_paths("combined")
p = lpa.HttpdLoglineParser("combined", fields)
for n in (100_000, 20_000):
    data = lpa.synth_combined(20261015, 0, n)
    r = p.parse_batch(data)
    print(n, r.counters, np.bincount(r.status, minlength=3)[:4], flush=True)
    buf, res = r.copy_to_host()
    cols = r.columns(res)
    st = cols[("status", 0)]
    print(" copy status", np.bincount(st, minlength=3)[:4], "arena_bytes", res.arena_bytes, "shard_cap", res.shard_cap, flush=True)
    bad = np.flatnonzero(st != 0)[:5]
    print(" first non-OK", bad, [data.split(b"\n")[i][:120] for i in bad], flush=True)
