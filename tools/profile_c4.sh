#!/bin/bash
# C4 (SASRec) evidence: GPU tests of the SASRec path, the bench line with its
# CPU baseline, and rocprofv3 kernel stats of the captured-graph step.
set -u
OUT=${PROF_OUT:-gpurun_out/prof_c4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sasrec or attention or resnorm or adam" > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python tools/bench_sasrec.py --steps 40 > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
grep '^{' $OUT/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/bench_sasrec.py --steps 10 --warmup 3 --cpu-baseline 0 > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo "trace ok"
