#!/bin/bash
# bf16x6 GEMM check: full GPU suite, GEMM shapes, C3 / C4 step lines.
set -u
export TMPDIR=/tmp
O=gpurun_out/x6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/gemm_bench.py > $O/gemm.jsonl 2> $O/gemm.err || { echo "gemm rc=$?"; exit 1; }
cat $O/gemm.jsonl
timeout -k 10 300 python tools/bench_sasrec.py --steps 100 --cpu-baseline 0 > $O/c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
grep '^{' $O/c4.log | cut -c1-300
timeout -k 10 300 python tools/bench_sage.py --steps 20 --cpu-baseline 0 > $O/c3.log 2>&1 || { echo "c3 rc=$?"; exit 1; }
grep '^{' $O/c3.log | cut -c1-300
REPS=20 timeout -k 10 200 python tools/dbg_rnbwd.py 2>&1 | grep "fused runs"
