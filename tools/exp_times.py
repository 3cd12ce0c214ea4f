"""Parse-kernel time of experiment builds (logparser_amd/_dbg/exp<N>.so) on
synthetic config-2 lines: python3 tools/exp_times.py LINES N1 N2 ... (0 = product)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n = int(sys.argv[1])
for e in sys.argv[2:]:
    env = dict(os.environ)
    if e != "0":
        env["LOGPARSER_AMD_LIB"] = os.path.join(ROOT, "logparser_amd", "_dbg", "exp%s.so" % e)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--lines", str(n), "--steps", "3",
                          "--warmup", "2", "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=400)
    try:
        d = json.loads(out.stdout.strip().splitlines()[-1])
        print("exp %s: parse %.3f ms index %.3f ms step %.3f ms" % (e, d["kernel_ms"]["parse_avg"], d["kernel_ms"]["index_avg"], d["ms_per_step"]), flush=True)
    except Exception:
        print("exp %s failed: %s" % (e, out.stderr[-500:]), flush=True)
