"""Print one step's device timeline from a rocprofv3 kernel trace: the
kernels from the last launch of a marker kernel (the step's first) to the
end of the trace, as (start us, idle gap before, duration, name).

    python tools/trace_step.py <kernel_trace.csv> [--marker bpr_sample_kernel] [--nth -1]"""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="bpr_sample_kernel")
    ap.add_argument("--nth", type=int, default=-1, help="which marker launch starts the step")
    ap.add_argument("--width", type=int, default=100)
    args = ap.parse_args()
    rows = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if re.search(args.marker, r[2])]
    i0 = marks[args.nth]
    i1 = marks[args.nth + 1] if args.nth + 1 < len(marks) and args.nth != -1 else len(rows)
    t0 = rows[i0][0]
    prev_end = t0
    busy = 0
    print(f"# {i1 - i0} kernels; start us, idle gap before, duration, kernel")
    for s, e, n in rows[i0:i1]:
        print(f"{(s - t0) / 1e3:9.1f} {max(0, s - prev_end) / 1e3:7.1f} {(e - s) / 1e3:7.1f} "
              f"{n[:args.width]}")
        busy += e - s
        prev_end = max(prev_end, e)
    print(f"# span {(prev_end - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
