# Round 4 (session 2n, after the host-path / owner-sum changes): kernel trace of the C3 world simulation at W = 8 with
# 2 micro-batches — where the device idles inside the pipelined step.
set -u
E=gpurun_out/r4s2
mkdir -p $E
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $E/prof -o run -- python3 tools/bench_world_sim.py --model sage --worlds 8 --exchanges fetch --microbatches 2 --steps 3 --warmup 2 > $E/sim.jsonl 2> $E/sim.log || { echo "rc=$?"; tail -5 $E/sim.log; exit 1; }
find $E/prof -name "*kernel_trace.csv" -exec cp {} $E/kernel_trace.csv \;
rm -rf $E/prof
python3 tools/trace_step_summary.py $E/kernel_trace.csv > $E/step_summary.txt && cat $E/step_summary.txt
