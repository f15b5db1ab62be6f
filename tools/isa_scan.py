"""List the device kernels of the built library that round an fp32 FMA straight to fp16
(v_fma_mixlo_f16 / v_fma_mixhi_f16 / v_mad_mixlo / v_mad_mixhi).

The reference computes every fp16 value it stores as an fp32 result rounded once more to half
(e.g. grid.h:148-162 weights, relative_l2.h:71 gradients, identity.h:59); the fused mix forms round
the unrounded FMA directly to fp16, which differs from fp32-then-fp16 in double-rounding cases.
The compiler forms them from fptrunc(fma) patterns, so tests/test_isa_rounding.py runs this over the
built library and requires an empty list.

  python tools/isa_scan.py [lib/libtcnn_mi355x.so]
"""
import os
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
MIX = ("v_fma_mixlo", "v_fma_mixhi", "v_mad_mixlo", "v_mad_mixhi")


def scan(lib):
    hits = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(d, "stripped")], check=True)
        b = open(fat, "rb").read()
        offs = []
        i = b.find(MAGIC)
        while i >= 0:
            offs.append(i)
            i = b.find(MAGIC, i + 1)
        for k, o in enumerate(offs):
            part, co = os.path.join(d, f"p{k}"), os.path.join(d, f"p{k}.co")
            open(part, "wb").write(b[o:offs[k + 1] if k + 1 < len(offs) else len(b)])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True, capture_output=True,
                                 text=True).stdout
            cur = None
            for line in dis.split("\n"):
                if line.endswith(">:"):
                    cur = line.split("<", 1)[1][:-2]
                elif any(m in line for m in MIX):
                    hits.setdefault(cur, []).append(line.strip())
    return hits, len(offs)


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                              "neuralbtf-tiny-cuda-nn_amd", "lib", "libtcnn_mi355x.so")
    hits, n = scan(lib)
    print(f"{n} code objects scanned")
    for k, v in hits.items():
        print(len(v), k)
        for l in v[:3]:
            print("   ", l)
