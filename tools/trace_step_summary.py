"""Summarise one pipelined step of a rocprofv3 kernel trace of
tools/bench_world_sim.py (the (k+1)-th bpr_sample_kernel starts step k):
device busy / idle time and the kernels by total time, per phase (before
the first micro-batch's forward, the micro-batches, after)."""
import csv
import re
import sys
from collections import defaultdict


def main(path, step=10):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    bs = [i for i, r in enumerate(rows) if "bpr_sample_kernel" in r["Kernel_Name"]]
    a, b = bs[step], bs[step + 1]
    t0 = int(rows[a]["Start_Timestamp"])
    prev, busy, idle = t0, 0, 0
    tot = defaultdict(float)
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        idle += max(0, s - prev)
        busy += e - s
        prev = max(prev, e)
        tot[re.sub(r"\(.*", "", r["Kernel_Name"])[-60:]] += (e - s) / 1e3
    print(f"span {(prev - t0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, idle {idle / 1e3:.1f} us")
    for k, v in sorted(tot.items(), key=lambda x: -x[1])[:30]:
        print(f"{v:8.1f} {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
