"""Summarise a tools/profile.sh run into profiles/ (committed evidence).

HBM bytes per dispatch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB (x1024); on gfx950 FETCH_SIZE reports half the bytes of
wide (16 B/lane) coalesced reads, so read bytes = 2 x FETCH_SIZE x 1024.
Every propagation read (float4 row gathers, col) is such a wide read.
"""
import csv
import glob
import json
import os
import shutil
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
tag = sys.argv[2] if len(sys.argv) > 2 else "r01"
workload = sys.argv[3] if len(sys.argv) > 3 else "C2-uniform-d64-L3"
os.makedirs("profiles", exist_ok=True)


def one(pattern):
    f = glob.glob(os.path.join(src, pattern), recursive=True)
    return f[0] if f else None


stats = one("trace/**/*kernel_stats.csv")
shutil.copy(stats, f"profiles/{tag}_kernel_stats.csv")
with open(stats) as f:
    rows = list(csv.DictReader(f))
summary = [{"kernel": r["Name"][:120], "calls": int(r["Calls"]),
            "avg_us": round(float(r["AverageNs"]) / 1e3, 2),
            "pct": float(r["Percentage"])} for r in rows]

per = {}
for kind in ("fetch", "write"):
    path = one(f"{kind}/**/*counter_collection.csv")
    with open(path) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"]
            d = per.setdefault(k, {"FETCH_SIZE": [], "WRITE_SIZE": []})
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    shutil.copy(path, f"profiles/{tag}_pmc_{kind}.csv")

kern = {}
for k, d in per.items():
    fs = sum(d["FETCH_SIZE"]) / max(len(d["FETCH_SIZE"]), 1)
    ws = sum(d["WRITE_SIZE"]) / max(len(d["WRITE_SIZE"]), 1)
    kern[k] = {"dispatches": len(d["FETCH_SIZE"]), "FETCH_SIZE_KiB": fs, "WRITE_SIZE_KiB": ws,
               "read_bytes": 2 * fs * 1024, "write_bytes": ws * 1024,
               "hbm_bytes_per_launch": 2 * fs * 1024 + ws * 1024}
dom = sys.argv[4] if len(sys.argv) > 4 else \
    "void mirec::prop_kernel<64, 4, 0, false, false>(mirec::PropK)"
out = {"workload": workload, "tag": tag, "kernel": dom,
       "hbm_bytes_per_launch": kern.get(dom, {}).get("hbm_bytes_per_launch"),
       "correction": "read = 2*FETCH_SIZE*1024 (gfx950 wide-read undercount), write = WRITE_SIZE*1024",
       "per_kernel": kern, "stats": summary[:12]}
with open("profiles/pmc_prop_kernel.json", "w") as f:
    json.dump(out, f, indent=1)
with open(f"profiles/{tag}_summary.json", "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps({k: {kk: (round(vv / 1e9, 3) if "bytes" in kk else vv) for kk, vv in v.items()}
                  for k, v in kern.items()}, indent=1))
for s in summary[:8]:
    print(s)
