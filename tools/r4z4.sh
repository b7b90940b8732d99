# Round 4 (session 2n): owner-side gather kernel — DP tests,
# host
# profile at 2 micro-batches, the C3 world simulation, the C3 line.
set -u
E=gpurun_out/r4z4
mkdir -p $E
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "owner_sum or scatter_rows or distinct_rows or export_stamped or pipelined or union or dp_trainer or routed or sage or table_grad" > $E/pytest.log 2>&1
rc=$?; tail -3 $E/pytest.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
timeout -k 10 300 python -u tools/host_profile_sage.py --chunks 2 > $E/host_c2.txt 2>&1 || { echo "rc=$?"; exit 1; }
timeout -k 10 600 python -u tools/bench_world_sim.py --model sage --worlds 1,8 --exchanges fetch,routed --microbatches 1,2,3,4 --steps 10 > $E/world_sim_c3.jsonl 2> $E/world_sim_c3.log || { echo "world sim rc=$?"; exit 1; }
timeout -k 10 300 python tools/bench_sage.py --steps 20 --cpu-baseline 0 > $E/bench_c3.log 2>&1 || { echo "bench rc=$?"; exit 1; }
head -2 $E/host_c2.txt | tail -1
grep '^{' $E/bench_c3.log | cut -c1-200
python3 -c "
import json
for l in open('$E/world_sim_c3.jsonl'):
    d=json.loads(l); p=d.get('projected') or {}
    print(d['world'], d['table_exchange'], d.get('microbatches'), d['ms_per_step_rank_compute'], d.get('chunk_compute_ms'), (p.get('300GBps') or {}))
"
