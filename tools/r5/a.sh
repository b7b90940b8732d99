# Round 5 (a): C4 gradient gate, C2 bench after the no-packed-f32 prop build,
# the DP launcher on one GPU with the real LightGCN, the micro-batch / DP /
# weighted-sampler tests.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5a
mkdir -p $E
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 500 --timeout-method thread -k "sasrec_c4_batch" > $E/pytest_c4.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -o "gradient rel err.*" $E/pytest_c4.log | cut -c1-5000; tail -3 $E/pytest_c4.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 500 --timeout-method thread -k "microbatch or dp_trainer_two_ranks or weighted_positive or sampler" > $E/pytest_mb.log 2>&1
rc=$?; echo "pytest mb rc=$rc"; tail -14 $E/pytest_mb.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > $E/bench_c2.log 2>&1 || { echo "bench rc=$?"; exit 1; }
grep '^{' $E/bench_c2.log | cut -c1-700
timeout -k 10 300 python -m furusato_recommend_amd.train_dp --model lgn --gpus 1 --synthetic 20000,2000,200000,cluster --recdim 64 --layer 3 --bpr_batch 4096 --epochs 2 --test_span 1 --train_iterative 1 --path $E/ck > $E/cli.log 2>&1 || { echo "cli rc=$?"; tail -20 $E/cli.log; exit 1; }
cut -c1-400 $E/cli.log | tail -5
for L in base tgA; do MIREC_LIB=var/libmirec_$L.so timeout -k 10 200 python tools/tg_bench.py --reps 50 >> $E/tg_ab.jsonl 2>> $E/tg_ab.log || { echo "tg_bench $L failed"; tail $E/tg_ab.log; exit 1; }; done
for L in base tgA; do MIREC_LIB=var/libmirec_$L.so timeout -k 10 200 python tools/tg_bench.py --reps 50 >> $E/tg_ab.jsonl 2>> $E/tg_ab.log || { echo "tg_bench $L failed"; exit 1; }; done
cat $E/tg_ab.jsonl
