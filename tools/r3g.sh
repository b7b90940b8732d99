# Round 3 evidence, part 1: whole GPU suite + smoke, then the C3 world
# simulation and the 2-rank DP rehearsals (gloo on one GPU).  Every GPU step
# has its own time limit; a failure ends the script.
set -u
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
O=gpurun_out/r3
run() {  # name, seconds, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run gpu_tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run world_sim_c3 400 python tools/bench_world_sim.py --model sage --worlds 1,2,4,8 --steps 10 --warmup 3
run c2_dp2_rehearse 300 python bench.py --gpus 2 --rehearse --steps 5 --warmup 2 --calib-steps 2
run sage_dp2_fetch 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29610 tools/bench_sage.py --rehearse --steps 5 --warmup 3 --table-exchange fetch --cpu-baseline 0
run sasrec_dp2 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 tools/bench_sasrec.py --rehearse --steps 5 --warmup 3 --cpu-baseline 0
