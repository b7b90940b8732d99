# Round 4 (session 2h): the fused table Adam with 2 (default) / 1 / 4 float4
# groups per thread and iteration — tests, then the C3 line per build (its
# live roofline times the Adam launch with HIP events) and the C4 line.
set -u
E=gpurun_out/r4l
mkdir -p $E
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "fused_table_adam or table_adam or sage_training_steps or sorted_table_step or c3_full_size or union_step" > $E/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $E/pytest.log | tail -2; if [ $rc -ne 0 ]; then exit $rc; fi
for v in libmirec var_adam_u1 var_adam_u4 libmirec var_adam_u1 var_adam_u4; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 200 python -u tools/bench_sage.py --cpu-baseline 0 > $E/c3_$v.json 2> $E/c3_$v.log
  rc=$?; echo "c3 $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('$E/c3_$v.json').readline()); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
timeout -k 10 300 python -u tools/bench_sasrec.py --cpu-baseline 0 > $E/c4.json 2> $E/c4.log
rc=$?; echo "c4 rc=$rc"; cut -c1-200 $E/c4.json
exit $rc
