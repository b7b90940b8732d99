# Round 5 (b): table-gradient A/B (base = round-4 pass 1, product = plan
# array), the C3 line, C5 on one GPU.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5b
mkdir -p $E
for rep in 1 2; do
  for L in base prod; do
    if [ $L = prod ]; then unset MIREC_LIB; else export MIREC_LIB=var/libmirec_$L.so; fi
    timeout -k 10 200 python tools/tg_bench.py --reps 50 > $E/tg_$L.json 2>> $E/tg_ab.log || { echo "tg_bench $L failed"; tail $E/tg_ab.log; exit 1; }
    echo "$L $(cat $E/tg_$L.json)" | tee -a $E/tg_ab.jsonl
  done
done
unset MIREC_LIB
timeout -k 10 400 python tools/bench_sage.py --steps 20 > $E/bench_c3.log 2>&1 || { echo "c3 rc=$?"; tail $E/bench_c3.log; exit 1; }
grep '^{' $E/bench_c3.log | cut -c1-400
timeout -k 10 900 python bench.py --users 10000000 --items 1000000 --edges 200000000 --dim 256 --steps 5 --warmup 2 --cpu-baseline off --quality-steps 0 --parity 0 > $E/bench_c5.log 2>&1 || { echo "c5 rc=$?"; tail $E/bench_c5.log; exit 1; }
grep '^{' $E/bench_c5.log | cut -c1-900
