"""Static guard for the gfx950 MFMA data hazards.

hipcc pads MFMA wait states only around instructions it generated; an inline-asm instruction that
reads an MFMA result too early (round 3: 76 GPU tests failed with garbage and run-to-run
differences) or writes an MFMA source operand one state before the MFMA (found by this test in the
round-3 library: the asm `v_pk_max_f16` ReLU fed MFMA B operands after 1 wait state where gfx950
needs 2, in 42 sites of the fused kernels) returns stale data on some waves of some launches, with
no error. tools/hazard_scan.py re-derives the rules from the disassembly of every kernel that issues
MFMAs, following the control flow; this test requires zero violations in the built library, and
first proves on a negative control (tests/isa/hazard_negative.hip) that the scanner catches both
kinds of site.
"""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd", "lib", "libtcnn_mi355x.so")
sys.path.insert(0, os.path.join(REPO, "tools"))

needs_llvm = pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"), reason="ROCm llvm tools missing")


@needs_llvm
@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc missing")
def test_scanner_catches_asm_hazards(tmp_path):
    import hazard_scan
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    obj = str(tmp_path / "neg.o")
    subprocess.run([hipcc, "--offload-arch=gfx950", "--cuda-device-only", "--no-gpu-bundle-output", "-O3", "-c",
                    os.path.join(REPO, "tests", "isa", "hazard_negative.hip"), "-o", obj], check=True)
    hits = hazard_scan.scan_disassembly(hazard_scan.disassemble_object(obj))
    rules = {name: {v[3] for v in vs} for name, vs in hits.items()}
    r1 = [n for n in rules if "r1" in n]
    r2 = [n for n in rules if "r2" in n]
    assert r1 and "R1" in rules[r1[0]], hits
    assert r2 and "R2" in rules[r2[0]], hits


@needs_llvm
@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_library_has_no_mfma_hazards():
    import hazard_scan
    hits, n = hazard_scan.scan(LIB)
    assert n >= 5, f"expected the library's device code objects, found {n}"
    assert not hits, {k: v[:3] for k, v in hits.items()}
