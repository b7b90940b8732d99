# Round 4 final tree, part 1: the whole GPU suite in one process.
set -u
export TMPDIR=/tmp
E=gpurun_out/r4z
mkdir -p $E
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rf --timeout 500 --timeout-method thread > $E/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $E/pytest.log
exit $rc
