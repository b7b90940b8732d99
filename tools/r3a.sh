set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "mf_c1 or users_rating or union_step or captured_step_equals or data_parallel or lgconv or dense_grad or score_topk or evaluate or routed" > gpurun_out/r3a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r3a_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --gpus 2 --rehearse --steps 5 --warmup 2 --calib-steps 2 > gpurun_out/r3a_rehearse.log 2>&1
rc=$?; echo "rehearse rc=$rc"; tail -3 gpurun_out/r3a_rehearse.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --quality-steps 0 --cpu-baseline off > gpurun_out/r3a_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/r3a_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python tools/eval_bench.py --users 10000000 --items 1000000 --edges 200000000 --dim 256 --reps 3 > gpurun_out/r3a_eval_c5.log 2>&1
rc=$?; echo "eval rc=$rc"; tail -4 gpurun_out/r3a_eval_c5.log
exit $rc
