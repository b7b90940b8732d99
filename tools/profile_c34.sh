#!/bin/bash
# rocprofv3 passes for the C3 (GraphSAGE) and C4 (SASRec) steps, each pass its
# own run (PMC passes with --pmc only, MI355X_MICROARCH.md §rocprofv3):
#   1. C3 --kernel-trace --stats
#   2. C4 --kernel-trace --stats
#   3. C4 SQ counters of the attention kernels (stall / LDS / MFMA breakdown)
set -u
OUT=${PROF_OUT:-gpurun_out/prof34}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/c3 -o run --output-format csv -- python3 tools/bench_sage.py --steps 10 --warmup 3 --cpu-baseline 0 > $OUT/c3.log 2>&1 || { echo "c3 trace rc=$?"; exit 1; }
echo "c3 trace ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/c4 -o run --output-format csv -- python3 tools/bench_sasrec.py --steps 10 --warmup 3 --cpu-baseline 0 > $OUT/c4.log 2>&1 || { echo "c4 trace rc=$?"; exit 1; }
echo "c4 trace ok"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex attn_ -d $OUT/c4sq -o run --output-format csv -- python3 tools/bench_sasrec.py --steps 3 --warmup 1 --cpu-baseline 0 > $OUT/c4sq.log 2>&1 || { echo "c4 sq pass rc=$?"; exit 1; }
echo "c4 sq ok"
