"""One-line summary of a bench.py log: value and per-kernel average durations."""
import json
import sys

for path in sys.argv[1:]:
    rec = None
    for line in open(path):
        if line.startswith("{"):
            rec = json.loads(line)
    if rec is None:
        print(path, "no JSON line")
        continue
    ks = " ".join(f"{k}={v['avg_us']:.1f}" for k, v in rec.get("kernels", {}).items() if v["share"] > 0.005)
    sp = rec.get("spmv", {})
    print(f"{path}: value={rec['value']:.1f} it/solve={rec.get('inner_iters_per_solve')} "
          f"spmv_us={sp.get('us', 0):.1f} ({sp.get('layout', '?')}, {sp.get('gbs', 0):.0f} GB/s) {ks}")
