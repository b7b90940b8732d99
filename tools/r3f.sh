# Round 3 (session 2): the col_sums fix — the new test, the captured / routed
# data-parallel tests and the SASRec / Linear tests.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "col_sums or linear or routed or captured or union_step or sasrec or dense_grad" > gpurun_out/r3f_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/r3f_pytest.log
exit $rc
