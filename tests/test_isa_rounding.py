"""Every fp16 value the kernels store from an fp32 result is rounded fp32-then-fp16, as the
reference's __float2half of an fp32 expression (grid.h:148-162 weights, relative_l2.h:71 gradients,
adam.h:114-123 weights, identity.h:59 outputs). hipcc folds fptrunc(fmul / fma / fsub) into
v_fma_mixlo/mixhi_f16, which rounds the exact result straight to fp16 and differs from the reference
whenever the fp32 rounding lands on an fp16 tie; csrc/common.h f16_rn blocks the fold where the
compiler would form it. This test disassembles the built library (the code objects in .hip_fatbin)
and requires that no kernel contains a mix-rounding instruction, so a compiler change that starts
folding a plain conversion shows up here instead of as a rare parity flake on the GPU.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd", "lib", "libtcnn_mi355x.so")
sys.path.insert(0, os.path.join(REPO, "tools"))


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="library or ROCm llvm tools missing")
def test_no_fused_mix_rounding_in_any_kernel():
    import isa_scan
    hits, n = isa_scan.scan(LIB)
    assert n >= 5, f"expected the library's device code objects, found {n}"
    assert not hits, {k: v[:2] for k, v in hits.items()}
