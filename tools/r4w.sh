# Round 4 (session 2n): host profile of the C3 GraphSAGE micro-batch with the
# backward on the calling thread (cProfile sees the backward functions).
set -u
E=gpurun_out/r4w
mkdir -p $E
timeout -k 10 300 python -u tools/host_profile_sage.py --chunks 2 --bwd-main-thread 1 --top 60 > $E/host_c2_main.txt 2>&1 || { echo "rc=$?"; tail -5 $E/host_c2_main.txt; exit 1; }
head -3 $E/host_c2_main.txt
