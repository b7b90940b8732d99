# Round 5: the C4 SASRec gradient test with the host-fp32 gate, verbose.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5a
mkdir -p $E
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 500 --timeout-method thread -k "sasrec_c4_batch" > $E/pytest_c4.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -o "gradient rel err.*" $E/pytest_c4.log | cut -c1-4000; tail -3 $E/pytest_c4.log
exit $rc
