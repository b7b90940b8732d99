# Round 5 (l): micro-batch trees sampled as the fetch planner reaches them
# (micro-batch 0's fetch overlaps the later trees' sampling): a fill micro
# bench, the DP / GraphSAGE tests, the C3 world simulation.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5l
mkdir -p $E
timeout -k 10 120 python tools/fill_bench.py || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 500 --timeout-method thread -k "dense_grad or pipelined or union or microbatch or sage" > $E/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAIL" $E/pytest.log | tail -15
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_world_sim.py --model sage --worlds 1,8 --exchanges fetch --microbatches 2,3 --steps 10 > $E/world_sim_c3.jsonl 2> $E/world_sim_c3.log || { echo "world sim rc=$?"; tail $E/world_sim_c3.log; exit 1; }
python3 -c "
import json
for l in open('$E/world_sim_c3.jsonl'):
    d=json.loads(l); print(d.get('microbatches'), d['ms_per_step_rank_compute'], d.get('plan_after_first_fetch_ms'), d.get('projected') and d['projected'].get('300GBps'))"
