# Round 3 (session 2): the whole GPU suite, smoke and the default bench line
# on the current tree.  Every GPU step has its own time limit.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r3e_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r3e_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3e_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r3e_smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/r3e_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/r3e_bench.log
exit $rc
