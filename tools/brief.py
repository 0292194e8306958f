"""Print one bench.py JSON line briefly: label, iterations, median solve ms, kernel classes."""
import json
import sys

for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        ks = {k: (v["avg_us"], v["launches"]) for k, v in d.get("kernels", {}).items()}
        print(sys.argv[2] if len(sys.argv) > 2 else "", d["inner_iters_per_solve"], round(d["solve_ms_median"], 3),
              round(d["value"], 1), ks)
