# Round 3: attention / SASRec tests after the pack-descriptor change, C3
# world simulation, DP rehearsals (gloo on one GPU), C3 / C4 single-GPU
# lines with BASELINE §3 CPU baselines, attention kernel timings.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r3b_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 gpurun_out/r3b_$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run tests_attn 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "attention or sasrec or packed or c3_full or shard"
run attn_bench 200 python tools/attn_bench.py --batches 2048 --mixes c4,64
run world_sim_c3 500 python tools/bench_world_sim.py --model sage --worlds 1,2,4,8 --steps 10 --warmup 3
run sage_dp2_fetch 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29610 tools/bench_sage.py --rehearse --steps 5 --warmup 3 --table-exchange fetch --cpu-baseline 0
run sage_dp2_routed 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 tools/bench_sage.py --rehearse --steps 5 --warmup 3 --table-exchange routed --cpu-baseline 0
run sage_dp2_dense 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 tools/bench_sage.py --rehearse --steps 5 --warmup 3 --table-exchange dense --cpu-baseline 0
run sasrec_dp2 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 tools/bench_sasrec.py --rehearse --steps 5 --warmup 3 --cpu-baseline 0
run bench_c3 500 python tools/bench_sage.py
run bench_c4 500 python tools/bench_sasrec.py
