# Round 4 (session 2n): onesweep from 128 K sort entries (the micro-batches'
# table-gradient sorts), the simulation handing the slice norms to the
# forward as dist does — table-gradient / GraphSAGE / DP tests, then the C3
# world simulation.
set -u
E=gpurun_out/r4t
mkdir -p $E
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "table_grad or sage or graphsage or pipelined or export_stamped or union or tg_" > $E/pytest.log 2>&1
rc=$?; tail -3 $E/pytest.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
timeout -k 10 600 python -u tools/bench_world_sim.py --model sage --worlds 1,8 --exchanges fetch,routed --microbatches 1,2,3,4 --steps 10 > $E/world_sim_c3.jsonl 2> $E/world_sim_c3.log || { echo "world sim rc=$?"; exit 1; }
timeout -k 10 300 python tools/bench_sage.py --steps 20 --cpu-baseline 0 > $E/bench_c3.log 2>&1 || { echo "bench rc=$?"; exit 1; }
grep '^{' $E/bench_c3.log | cut -c1-300
python3 -c "
import json
for l in open('$E/world_sim_c3.jsonl'):
    d=json.loads(l); p=d.get('projected') or {}
    print(d['world'], d['table_exchange'], d.get('microbatches'), d['ms_per_step_rank_compute'], d.get('chunk_compute_ms'), (p.get('300GBps') or {}))
"
