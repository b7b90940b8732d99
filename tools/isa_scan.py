"""Scan the gfx950 code of a built library for the instruction shape behind
the fused dX + LayerNorm-backward kernel's wrong rows: a
packed-f32 VALU op (v_pk_*_f32) whose op_sel makes its LOW lane read the
HIGH dword of a register pair, in a kernel that also issues MFMAs
(tools/op_sel_repro.hip reproduces wrong upper-lane reads of exactly that
shape after MFMA work).

    python tools/isa_scan.py [furusato_recommend_amd/libmirec.so]

Prints, per kernel with such reads, (MFMA count, read count, name); exits 1
when a kernel has both.  The library's .hip_fatbin holds one offload bundle
per translation unit; each is unbundled for gfx950 and disassembled with the
ROCm llvm tools (no GPU needed)."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
OPSEL_HI = re.compile(r"v_pk_\w+_f32\b.*\bop_sel:\[[01,]*1")


def kernels(so: str) -> dict:
    """{kernel symbol: {"mfma": count, "opsel_hi": [instructions]}}"""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", so,
                        os.devnull], check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
        for k in range(len(starts) - 1):
            bundle, co = os.path.join(td, f"b{k}"), os.path.join(td, f"c{k}.o")
            with open(bundle, "wb") as f:
                f.write(data[starts[k]:starts[k + 1]])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                            f"--input={bundle}", f"--targets={TARGET}", f"--output={co}"],
                           check=True, capture_output=True)
            txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co],
                                 capture_output=True, text=True, check=True).stdout
            fn = None
            for line in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
                if m:
                    fn = m.group(1)
                    out.setdefault(fn, {"mfma": 0, "opsel_hi": []})
                elif fn is not None:
                    if "v_mfma" in line:
                        out[fn]["mfma"] += 1
                    if OPSEL_HI.search(line):
                        out[fn]["opsel_hi"].append(line.strip())
    return out


def hazards(so: str) -> list:
    """Kernels with MFMAs AND low-lane high-dword op_sel reads."""
    return sorted(fn for fn, v in kernels(so).items() if v["mfma"] and v["opsel_hi"])


if __name__ == "__main__":
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
        "furusato_recommend_amd", "libmirec.so")
    ks = kernels(so)
    for fn, v in sorted(ks.items()):
        if v["opsel_hi"]:
            print(v["mfma"], len(v["opsel_hi"]), fn)
    bad = hazards(so)
    print(f"{len(ks)} kernels, {sum(1 for v in ks.values() if v['mfma'])} with MFMA, "
          f"{sum(1 for v in ks.values() if v['opsel_hi'])} with high-dword op_sel reads, "
          f"{len(bad)} with both")
    sys.exit(1 if bad else 0)
