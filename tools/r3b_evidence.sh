#!/bin/bash
# Round-3 (second half) evidence for the bf16x6 GEMMs: C3 / C4 bench lines
# with their CPU baselines, rocprof kernel stats of both, GEMM shapes.
set -u
export TMPDIR=/tmp
E=gpurun_out/r3b
mkdir -p $E
timeout -k 10 300 python tools/bench_sage.py --steps 20 > $E/bench_c3.log 2>&1 || { echo "c3 rc=$?"; exit 1; }
grep '^{' $E/bench_c3.log | cut -c1-200
timeout -k 10 300 python tools/bench_sasrec.py --steps 100 > $E/bench_c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
grep '^{' $E/bench_c4.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/c3 -o run --output-format csv -- python3 tools/bench_sage.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/c3.log 2>&1 || { echo "c3 trace rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/c4 -o run --output-format csv -- python3 tools/bench_sasrec.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/c4.log 2>&1 || { echo "c4 trace rc=$?"; exit 1; }
timeout -k 10 200 python tools/gemm_bench.py > $E/gemm.jsonl 2> $E/gemm.err || { echo "gemm rc=$?"; exit 1; }
echo "evidence ok"
