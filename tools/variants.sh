#!/bin/bash
# A/B timing of engine switches (tools/bench_variants.py) under a time limit.
set -u
mkdir -p gpurun_out
timeout -k 10 ${VAR_T:-500} python tools/bench_variants.py ${VAR_ARGS:-} > gpurun_out/variants.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/variants.log | tail -20
exit $rc
