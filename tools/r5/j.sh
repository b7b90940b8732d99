# Round 5 (j): device timeline of one simulated C3 pipelined step (W = 8,
# C = 2) under rocprofv3 --kernel-trace.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5j
mkdir -p $E
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $E/tr -o run -- python3 tools/bench_world_sim.py --model sage --worlds 8 --exchanges fetch --microbatches 2 --steps 3 --warmup 2 > $E/sim.log 2>&1 || { echo "rc=$?"; tail $E/sim.log; exit 1; }
f=$(find $E/tr -name '*kernel_trace.csv' | head -1)
python3 tools/trace_step.py $f --width 110 > $E/step.txt
cp $f $E/kernel_trace.csv
rm -rf $E/tr
wc -l $E/step.txt; tail -3 $E/step.txt
