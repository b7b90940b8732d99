# Round 5 (k): the row movers (gather / counted gather / scatter / owner sum
# with four rows or blocks in flight per lane): their tests, the GraphSAGE
# and data-parallel tests, then the C3 world simulation at W = 1, 8.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5k
mkdir -p $E
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 500 --timeout-method thread -k "row_movers or scatter_rows or owner_sum or distinct_rows or dense_grad or pipelined or union or microbatch or sage or graphsage" > $E/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAIL" $E/pytest.log | tail -15
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_world_sim.py --model sage --worlds 1,8 --exchanges fetch --microbatches 2,3 --steps 10 > $E/world_sim_c3.jsonl 2> $E/world_sim_c3.log || { echo "world sim rc=$?"; tail $E/world_sim_c3.log; exit 1; }
cut -c1-700 $E/world_sim_c3.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $E/tr -o run -- python3 tools/bench_world_sim.py --model sage --worlds 8 --exchanges fetch --microbatches 2 --steps 3 --warmup 2 > $E/sim_tr.log 2>&1 || { echo "rc=$?"; tail $E/sim_tr.log; exit 1; }
f=$(find $E/tr -name '*kernel_trace.csv' | head -1)
cp $f $E/kernel_trace.csv
rm -rf $E/tr
