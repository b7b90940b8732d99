# The C3 world simulation (W = 1 baseline, W = 8 pipelined with two
# micro-batches) run twice in each timing mode on one box: per-step
# synchronisation (the default) and --no-step-sync.  The spread between
# runs of the same mode is the box's noise on this host-launch-bound step.
#   gpurun -- 'bash tools/c3_repeat.sh'  -> gpurun_out/c3rep/{sync,nosync}_{1,2}.jsonl
set -e
O=gpurun_out/c3rep
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u tools/bench_world_sim.py --model sage --worlds 1,8 --exchanges fetch --microbatches 2 --steps 30 > $O/sync_$i.jsonl 2> $O/sync_$i.log
  timeout -k 10 300 python -u tools/bench_world_sim.py --model sage --worlds 1,8 --exchanges fetch --microbatches 2 --steps 30 --no-step-sync > $O/nosync_$i.jsonl 2> $O/nosync_$i.log
done
