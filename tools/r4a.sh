# Round 4 (session 1): the two non-determinism investigations, the captured
# DP fix, and the bench line with the in-run oracle parity.
set -u
mkdir -p gpurun_out/r4a
export TMPDIR=/tmp
for v in libmirec var_cur_masked var_old_clamped var_old_masked var_old_masked_wz; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so REPS=20 timeout -k 10 200 python -u tools/dbg_rnbwd.py > gpurun_out/r4a/rnbwd_$v.log 2>&1
  rc=$?; echo "rnbwd $v rc=$rc"; grep "fused runs" gpurun_out/r4a/rnbwd_$v.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
REPS=200 timeout -k 10 300 python -u tools/dbg_colsum_graph.py > gpurun_out/r4a/colsum.jsonl 2>&1
rc=$?; echo "colsum rc=$rc"; cat gpurun_out/r4a/colsum.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -k "captured_step_equals_eager or dp_trainer or c4_batch_step or distinct_rows or repeatable or pipelined or evaluate_matches or score_topk" > gpurun_out/r4a/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/r4a/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 700 python bench.py > gpurun_out/r4a/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/r4a/bench.log
exit $rc
