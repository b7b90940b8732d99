# Round 5 (o): 1-block sequences riding in the 3-block packs of the packed
# attention backward: attention / SASRec tests, attn_bench at the C4 mix,
# the C4 line.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5o
mkdir -p $E
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 500 --timeout-method thread -k "attention or sasrec or attn" > $E/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAIL|Error" $E/pytest.log | tail -8
[ $rc = 0 ] || exit $rc
timeout -k 10 120 python tools/attn_bench.py --mixes c4 --batches 2048 --reps 20 > $E/attn.jsonl 2>&1 || { echo "bench rc=$?"; tail $E/attn.jsonl; exit 1; }
grep -E "packed_bwd|wave_fwd" $E/attn.jsonl
timeout -k 10 400 python -u tools/bench_sasrec.py --steps 100 > $E/c4.log 2>&1 || { echo "c4 rc=$?"; tail $E/c4.log; exit 1; }
grep '^{' $E/c4.log | cut -c1-600
