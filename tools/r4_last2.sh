# Round 4, very last tree: the whole GPU suite.
set -u
export TMPDIR=/tmp
E=gpurun_out/r4last2
mkdir -p $E
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 500 --timeout-method thread > $E/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $E/pytest.log
exit $rc
