"""Per-step-index band-step table from a bench.py log run with VTK_PROF_PERJ=1:
j, launches, avg us, algorithmic GB/s and fraction of 8 TB/s."""
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
    print(f"{path}: value={rec['value']:.1f} it/s")
    rows = sorted((k, v) for k, v in rec.get("kernels", {}).items() if k.startswith("band_step_j"))
    for k, v in rows:
        print(f"  {k[-3:]}  {v['launches']:4d}  {v['avg_us']:8.1f} us  {v['gbs']:7.1f} GB/s  {v['gbs'] / 8000:.3f}")
    others = {k: v for k, v in rec.get("kernels", {}).items() if not k.startswith("band_step_j") and v["share"] > 0.003}
    print("  other:", " ".join(f"{k}={v['avg_us']:.1f}us" for k, v in others.items()))
