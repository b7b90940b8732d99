# Round 4 (session 2m): GraphSAGE table-row gather with 4 rows per thread in
# flight — the GraphSAGE tests, then C3 per build (line + kernel times)
# against the tree before it (var_sage_prev).
set -u
E=gpurun_out/r4q
mkdir -p $E
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "sage or fanout" > $E/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $E/pytest.log | tail -2; if [ $rc -ne 0 ]; then exit $rc; fi
for v in libmirec var_sage_prev libmirec var_sage_prev; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 200 python -u tools/bench_sage.py --cpu-baseline 0 > $E/c3_$v.json 2> $E/c3_$v.log
  rc=$?; echo "c3 $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  python3 -c "import json; d=json.loads(open('$E/c3_$v.json').readline()); print('$v', d['ms_per_step'])"
done
for v in libmirec var_sage_prev; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $E/prof_$v -o run -- python3 tools/bench_sage.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/prof_$v.log 2>&1
  rc=$?; echo "prof $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
find $E -name "*kernel_trace.csv" -delete
for v in libmirec var_sage_prev; do echo "== $v"; f=$(find $E/prof_$v -name "*kernel_stats.csv"); grep -E "fanout|gather_rows" "$f" | cut -d, -f1-4 | sed 's/(.*"//'; done
