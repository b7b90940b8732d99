#!/bin/bash
# HBM bytes of the C3 table Adam (tg_adam_kernel): FETCH_SIZE and WRITE_SIZE
# passes, each its own run (MI355X_MICROARCH.md §HBM; gfx950 correction:
# read = 2 x FETCH_SIZE x 1024, write = WRITE_SIZE x 1024).
set -u
export TMPDIR=/tmp
O=gpurun_out/pmc_adam
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex tg_adam -d $O/fetch -o run --output-format csv -- python3 tools/bench_sage.py --steps 5 --warmup 2 --cpu-baseline 0 > $O/fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex tg_adam -d $O/write -o run --output-format csv -- python3 tools/bench_sage.py --steps 5 --warmup 2 --cpu-baseline 0 > $O/write.log 2>&1 || { echo "write rc=$?"; exit 1; }
echo "pmc ok"
