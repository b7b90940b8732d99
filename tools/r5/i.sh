# Round 5 (i): GraphSAGE DP with the row fetches on their own communicator
# (micro-batch 0's fetch issued before the later read sets are planned): the
# data-parallel tests, then the C3 world simulation at W = 1, 8.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5i
mkdir -p $E
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 500 --timeout-method thread -k "dense_grad or pipelined or union or microbatch" > $E/pytest_dp.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|PASS|FAIL" $E/pytest_dp.log | tail -25
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_world_sim.py --model sage --worlds 1,8 --exchanges fetch --microbatches 2,3 --steps 10 > $E/world_sim_c3.jsonl 2> $E/world_sim_c3.log || { echo "world sim rc=$?"; tail $E/world_sim_c3.log; exit 1; }
cut -c1-900 $E/world_sim_c3.jsonl
