#!/bin/bash
# A/B of the attention kernels inside the C4 step: kernel durations from
# rocprofv3 (host-bound steps make event timings include launch gaps).
set -u
OUT=gpurun_out/ab_attn
mkdir -p $OUT
export TMPDIR=/tmp
for b in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/b$b -o run --output-format csv -- python3 tools/bench_sasrec.py --steps 10 --warmup 3 --cpu-baseline 0 --attn-buckets $b > $OUT/b$b.log 2>&1 || { echo "b$b rc=$?"; exit 1; }
done
python3 - <<'PY'
import csv, collections
for b in (1, 0):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(f"gpurun_out/ab_attn/b{b}/run_kernel_stats.csv")):
        if "attn_" in r["Name"]:
            k = "fwd" if "fwd" in r["Name"] else "bwd"
            agg[k][0] += int(r["Calls"]); agg[k][1] += float(r["TotalDurationNs"])
    print("buckets", b, {k: round(v[1] / 1e3 / 26, 1) for k, v in agg.items()}, "us per call (26 calls)")
PY
