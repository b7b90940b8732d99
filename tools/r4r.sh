# Round 4 (session 2n): device-side export of the micro-batches' table-gradient
# rows (export_stamped) with the route deferred one micro-batch — its tests,
# the pipelined / union DP tests, then the C3 world simulation.
set -u
E=gpurun_out/r4r
mkdir -p $E
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "export_stamped or distinct_rows or pipelined or union_step or dp_trainer or routed" > $E/pytest.log 2>&1
rc=$?; tail -3 $E/pytest.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
timeout -k 10 600 python -u tools/bench_world_sim.py --model sage --worlds 1,8 --exchanges fetch --microbatches 1,2,4 --steps 10 > $E/world_sim_c3.jsonl 2> $E/world_sim_c3.log || { echo "world sim rc=$?"; exit 1; }
cat $E/world_sim_c3.jsonl
