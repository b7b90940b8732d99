#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench.  Every GPU step has
# its own time limit; a crash / timeout (rc not in {0,1}) ends the session.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${PYTEST_T:-900} python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 ${BENCH_T:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
