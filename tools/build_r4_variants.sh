#!/bin/bash
# Round-4 A/B libraries (furusato_recommend_amd/var_*.so, selected with
# MIREC_LIB): every object of the current tree except the one varied.
#   var_cur_masked     gemm.hip with exec-masked row-tail loads (MIREC_RNBWD_MASKED=1)
#   var_cur_masked_wz  the same built with -amdgpu-waitcnt-forcezero
#   var_cur_masked_w0  masked + s_waitcnt 0 after the row loads (=2)
#   var_cur_masked_stats / _rows  only the statistics / only the rows masked (=3 / =4)
#   var_old_masked     gemm.hip of commit cee0a0b (round 3, wave-side split loop)
#                      with its original exec-masked loads — the failing form
#   var_old_masked_wz  the same built with -amdgpu-waitcnt-forcezero
#   var_old_clamped    gemm.hip of commit cee0a0b as committed (clamped loads)
#   var_topk_f32       topk.hip with the f32 score tiles (MIREC_TOPK_X6=0)
set -e
cd $(dirname $0)/..
make -s -C furusato_recommend_amd/csrc
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Iinclude -Wall -Wno-unused-result --offload-arch=gfx950 -munsafe-fp-atomics"
T=build/var/old
mkdir -p $T
git show cee0a0b:furusato_recommend_amd/csrc/gemm.hip > $T/gemm.hip
git show cee0a0b:furusato_recommend_amd/csrc/common.h > $T/common.h
python3 - "$T/gemm.hip" "$T/gemm_masked.hip" <<'EOF'
import sys
s = open(sys.argv[1]).read()
old = """    const int64_t r = min(m0 + g + 8 * q, n - 1);
    ov[q] = ld4(a.out + r * kTile + c);
    gv[q] = a.g_out ? ld4(a.g_out + r * kTile + c) : f4_zero();
    mv[q] = a.mean[r];
    sv[q] = a.rstd[r];"""
new = """    const int64_t r = m0 + g + 8 * q;
    const bool ok = r < n;
    ov[q] = ok ? ld4(a.out + r * kTile + c) : f4_zero();
    gv[q] = (ok && a.g_out) ? ld4(a.g_out + r * kTile + c) : f4_zero();
    mv[q] = ok ? a.mean[r] : 0.f;
    sv[q] = ok ? a.rstd[r] : 0.f;"""
assert s.count(old) == 1
open(sys.argv[2], "w").write(s.replace(old, new))
EOF
$H -DMIREC_RNBWD_MASKED=1 -c furusato_recommend_amd/csrc/gemm.hip -o build/var/cur_masked.o &
$H -DMIREC_RNBWD_MASKED=1 -mllvm -amdgpu-waitcnt-forcezero -c furusato_recommend_amd/csrc/gemm.hip -o build/var/cur_masked_wz.o &
$H -DMIREC_RNBWD_MASKED=2 -c furusato_recommend_amd/csrc/gemm.hip -o build/var/cur_masked_w0.o &
$H -DMIREC_RNBWD_MASKED=3 -c furusato_recommend_amd/csrc/gemm.hip -o build/var/cur_masked_stats.o &
$H -DMIREC_RNBWD_MASKED=4 -c furusato_recommend_amd/csrc/gemm.hip -o build/var/cur_masked_rows.o &
$H -c $T/gemm_masked.hip -o build/var/old_masked.o &
$H -mllvm -amdgpu-waitcnt-forcezero -c $T/gemm_masked.hip -o build/var/old_masked_wz.o &
$H -c $T/gemm.hip -o build/var/old_clamped.o &
$H -DMIREC_TOPK_X6=0 -c furusato_recommend_amd/csrc/topk.hip -o build/var/topk_f32.o &
wait
link() {  # name, replaced object, variant object
  objs=$(ls build/obj/*.o | grep -v "/$2.o\$")
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $3 -lpthread -o furusato_recommend_amd/$1.so
}
link var_cur_masked gemm build/var/cur_masked.o
link var_cur_masked_wz gemm build/var/cur_masked_wz.o
link var_cur_masked_w0 gemm build/var/cur_masked_w0.o
link var_cur_masked_stats gemm build/var/cur_masked_stats.o
link var_cur_masked_rows gemm build/var/cur_masked_rows.o
link var_old_masked gemm build/var/old_masked.o
link var_old_masked_wz gemm build/var/old_masked_wz.o
link var_old_clamped gemm build/var/old_clamped.o
link var_topk_f32 topk build/var/topk_f32.o
ls -la furusato_recommend_amd/var_*.so
