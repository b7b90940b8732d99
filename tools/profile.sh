#!/bin/bash
# rocprofv3 passes for the bench workload (each pass its own run, PMC passes
# with --pmc only, per MI355X_MICROARCH.md §rocprofv3 / §HBM):
#   1. --kernel-trace --stats  -> per-kernel average durations
#   2. --pmc FETCH_SIZE        -> HBM read bytes per dispatch (KB; x2 on gfx950 for wide reads)
#   3. --pmc WRITE_SIZE        -> HBM write bytes per dispatch (KB)
set -u
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
export TMPDIR=/tmp
BARGS=${BENCH_ARGS:-"--steps 10 --warmup 3 --cpu-baseline off --quality-steps 0 --parity 0"}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $BARGS > $OUT/trace.log 2>&1 || { echo "trace pass rc=$?"; exit 1; }
echo "trace ok"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex prop_kernel -d $OUT/fetch -o run --output-format csv -- python3 bench.py $BARGS > $OUT/fetch.log 2>&1 || { echo "fetch pass rc=$?"; exit 1; }
echo "fetch ok"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex prop_kernel -d $OUT/write -o run --output-format csv -- python3 bench.py $BARGS > $OUT/write.log 2>&1 || { echo "write pass rc=$?"; exit 1; }
echo "write ok"
