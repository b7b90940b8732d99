# Round 4 (session 2k): C5 on one GPU and the C2 Zipf graph with the final
# tree (prop_finalize / BPR kernels now built without packed-f32 ops).
set -u
E=gpurun_out/r4o
mkdir -p $E
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --kind zipf --steps 20 --warmup 5 --cpu-baseline off --quality-steps 0 --parity 0 > $E/bench_c2_zipf.log 2>&1
rc=$?; echo "zipf rc=$rc"; grep '^{' $E/bench_c2_zipf.log | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 700 python bench.py --users 10000000 --items 1000000 --edges 200000000 --dim 256 --steps 5 --warmup 2 --cpu-baseline off --quality-steps 0 --parity 0 > $E/bench_c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; grep '^{' $E/bench_c5.log | cut -c1-300
exit $rc
