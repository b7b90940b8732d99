# Round 4: narrowing the masked-load failure of the fused dX + LayerNorm-
# backward kernel (which loads, and whether draining the counters fixes it),
# the C4 oracle test with diagnostics, the DP driver tests, the C2 bench line
# with its oracle parity leg.
set -u
mkdir -p gpurun_out/r4d
export TMPDIR=/tmp
for v in var_cur_masked_w0 var_cur_masked_wz var_cur_masked_stats var_cur_masked_rows; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so REPS=20 timeout -k 10 200 python -u tools/dbg_rnbwd.py > gpurun_out/r4d/rnbwd_$v.log 2>&1
  rc=$?; echo "rnbwd $v rc=$rc"; grep "fused runs" gpurun_out/r4d/rnbwd_$v.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -k "c4_batch_step or dp_trainer" > gpurun_out/r4d/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r4d/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python bench.py > gpurun_out/r4d/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3500 gpurun_out/r4d/bench.log
exit $rc
