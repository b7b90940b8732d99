#!/bin/bash
# N-rank code paths on one GPU (gloo collectives, every rank on cuda:0): the
# C2 bench at 8 ranks (auto calibration, sharded chunks), C3 / C4 at 4 ranks.
set -u
export TMPDIR=/tmp
E=gpurun_out/rh
mkdir -p $E
timeout -k 10 900 python bench.py --gpus 8 --rehearse --steps 3 --warmup 2 --quality-steps 0 --cpu-baseline off > $E/c2_dp8.log 2>&1 || { echo "c2 dp8 rc=$?"; tail -20 $E/c2_dp8.log; exit 1; }
grep '^{' $E/c2_dp8.log | cut -c1-300
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 tools/bench_sage.py --rehearse --steps 3 --warmup 2 --cpu-baseline 0 > $E/c3_dp4.log 2>&1 || { echo "c3 dp4 rc=$?"; tail -20 $E/c3_dp4.log; exit 1; }
grep '^{' $E/c3_dp4.log | cut -c1-300
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 tools/bench_sasrec.py --rehearse --steps 3 --warmup 2 --cpu-baseline 0 > $E/c4_dp4.log 2>&1 || { echo "c4 dp4 rc=$?"; tail -20 $E/c4_dp4.log; exit 1; }
grep '^{' $E/c4_dp4.log | cut -c1-300
echo "rehearsal ok"
