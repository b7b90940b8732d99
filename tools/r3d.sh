set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "captured_step_equals or shard_pack" > gpurun_out/r3d_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r3d_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --gpus 2 --rehearse --steps 5 --warmup 2 --calib-steps 2 > gpurun_out/r3a_rehearse.log 2>&1
rc=$?; echo "rehearse rc=$rc"; tail -3 gpurun_out/r3a_rehearse.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --quality-steps 0 --cpu-baseline off > gpurun_out/r3a_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/r3a_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python tools/eval_bench.py --users 10000000 --items 1000000 --edges 200000000 --dim 256 --reps 3 > gpurun_out/r3a_eval_c5.log 2>&1
rc=$?; echo "eval rc=$rc"; tail -4 gpurun_out/r3a_eval_c5.log
exit $rc
