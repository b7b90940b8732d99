# Round 4 (session 2n): host-side profile of the C3 GraphSAGE step, whole
# batch and as 2 micro-batches.
set -u
E=gpurun_out/r4u
mkdir -p $E
timeout -k 10 300 python -u tools/host_profile_sage.py --chunks 1 > $E/host_c1.txt 2>&1 || { echo "rc=$?"; tail -5 $E/host_c1.txt; exit 1; }
timeout -k 10 300 python -u tools/host_profile_sage.py --chunks 2 > $E/host_c2.txt 2>&1 || { echo "rc=$?"; tail -5 $E/host_c2.txt; exit 1; }
head -3 $E/host_c1.txt; head -3 $E/host_c2.txt
