"""VGPR / AGPR / scratch / LDS of the library's kernels whose mangled name contains a pattern
(from the code-object metadata notes of the .hip_fatbin bundles).

  python tools/kernel_resources.py k_grid_bwd_lds      (TCNN_LIB_PATH: another build of the library)
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(lib, d):
    fat = os.path.join(d, "fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(d, "stripped")], check=True)
    b = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    offs = [m.start() for m in re.finditer(re.escape(magic), b)]
    out = []
    for k, o in enumerate(offs):
        part, co = os.path.join(d, f"p{k}"), os.path.join(d, f"p{k}.co")
        open(part, "wb").write(b[o:offs[k + 1] if k + 1 < len(offs) else len(b)])
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        out.append(co)
    return out


def main():
    pat = sys.argv[1] if len(sys.argv) > 1 else ""
    lib = os.environ.get("TCNN_LIB_PATH") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                          "neuralbtf-tiny-cuda-nn_amd", "lib", "libtcnn_mi355x.so")
    keys = (".vgpr_count", ".agpr_count", ".private_segment_fixed_size", ".group_segment_fixed_size", ".vgpr_spill_count")
    with tempfile.TemporaryDirectory() as d:
        for co in code_objects(lib, d):
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
            # one kernel per "- .agpr_count" record; the record holds .name
            for rec in notes.split("  - .agpr_count")[1:]:
                rec = ".agpr_count" + rec
                m = re.search(r"\.name:\s+(\S+)", rec)
                if not m or pat not in m.group(1):
                    continue
                vals = {k: (re.search(re.escape(k) + r":\s+(\d+)", rec) or [None, "?"])[1] for k in keys}
                print(m.group(1)[:110], " ".join(f"{k[1:]}={v}" for k, v in vals.items()))


if __name__ == "__main__":
    main()
