set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "union_step and sasrec" > gpurun_out/r3dbg.log 2>&1
echo rc=$?; grep -n "AssertionError: {" gpurun_out/r3dbg.log | cut -c1-600
exit 0
