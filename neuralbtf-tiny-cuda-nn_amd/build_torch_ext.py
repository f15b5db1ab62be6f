"""Build the torch autograd node of tinycudann.Module (csrc/torch_ext.cpp) in-tree:
lib/_tcnn_torch<EXT_SUFFIX>, host-only C++ against the installed torch and lib/libtcnn_mi355x.so
(g++ directly; ~50 s). Called by __graft_entry__.build(); rebuilds only when a source is newer."""
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))


def target():
    return os.path.join(HERE, "lib", "_tcnn_torch" + sysconfig.get_config_var("EXT_SUFFIX"))


def build(force=False):
    import torch
    from torch.utils import cpp_extension as ce
    src = os.path.join(HERE, "csrc", "torch_ext.cpp")
    deps = [src, os.path.join(HERE, "..", "include", "tcnn_mi355x.h"), os.path.join(HERE, "lib", "libtcnn_mi355x.so")]
    out = target()
    if not force and os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return out
    cmd = ["g++", "-O2", "-shared", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
           "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM", "-DTORCH_EXTENSION_NAME=_tcnn_torch", "-DTORCH_API_INCLUDE_EXTENSION_H"]
    for p in ce.include_paths():
        cmd += ["-I", p]
    cmd += ["-I", sysconfig.get_paths()["include"], "-isystem", "/opt/rocm/include", src]
    for p in ce.library_paths():
        cmd += ["-L", p, f"-Wl,-rpath,{p}"]
    cmd += ["-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-L", os.path.join(HERE, "lib"), "-ltcnn_mi355x",
            "-Wl,-rpath,$ORIGIN", "-o", out]
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
