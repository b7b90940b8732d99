#!/bin/bash
# rocprofv3 kernel stats of the C4 step (graph mode) with the given env, and
# a per-kernel-family summary (ms per step over the 13 captured steps).
set -u
OUT=gpurun_out/c4s_${1:-x}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 tools/bench_sasrec.py --steps 10 --warmup 3 --cpu-baseline 0 > $OUT/log 2>&1 || { echo "rc=$?"; exit 1; }
python3 - $OUT <<'PY'
import csv, re, sys, collections
fam = collections.Counter()
for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_stats.csv")):
    n = r["Name"]
    k = ("Cijk(blas)" if n.startswith("Cijk") else re.sub(r"[<(].*", "", n).replace("void ", "")[:50])
    fam[k] += float(r["TotalDurationNs"]) / 1e6 / 18
for k, v in fam.most_common(22):
    print(f"{v:7.3f} ms/step  {k}")
print("total", round(sum(fam.values()), 3))
PY
