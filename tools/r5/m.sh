# Round 5 (m): the table gradient's packed export (mirec_table_grad_sorted_rows)
# in the pipelined exchange, kept have-map: table-gradient / DP / GraphSAGE
# tests, the C3 world simulation (W = 1 timed over 30 steps).
set -u
export TMPDIR=/tmp
E=gpurun_out/r5m
mkdir -p $E
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 500 --timeout-method thread -k "table_grad or dense_grad or pipelined or union or microbatch or sage or row_movers or owner_sum" > $E/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAIL|Error" $E/pytest.log | tail -15
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_world_sim.py --model sage --worlds 1,8 --exchanges fetch --microbatches 2,3 --steps 30 > $E/world_sim_c3.jsonl 2> $E/world_sim_c3.log || { echo "world sim rc=$?"; tail $E/world_sim_c3.log; exit 1; }
python3 -c "
import json
for l in open('$E/world_sim_c3.jsonl'):
    d=json.loads(l); print(d.get('microbatches'), d['ms_per_step_rank_compute'], d.get('chunk_compute_ms'), d.get('plan_after_first_fetch_ms'), d.get('projected') and d['projected'].get('300GBps'))"
