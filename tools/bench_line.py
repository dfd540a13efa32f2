"""Print value (M/s), ms/step and the parity verdict of a bench.py JSON line file."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d.get("parity") or {}
print("%.2f M/s %.3f ms parity %s" % (d["value"] / 1e6, d["ms_per_step"], p.get("pass")))
