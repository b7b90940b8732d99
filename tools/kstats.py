"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv.

    python tools/kstats.py gpurun_out/prof/run_kernel_stats.csv [--steps N] [--top K]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
ap.add_argument("--top", type=int, default=20)
ap.add_argument("--match", default="")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.csv)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
    if a.match and a.match not in r["Name"]:
        continue
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}% calls={r['Calls']:>5} "
          f"avg={float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:100]}")
print(f"total {tot / 1e6:.3f} ms" + (f", {tot / 1e6 / a.steps:.3f} ms/step" if a.steps else ""))
