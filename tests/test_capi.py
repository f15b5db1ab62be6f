"""CPU checks of the C-ABI boundary: the HIP library loads (no GPU needed to dlopen) and exports
every entry point include/tcnn_mi355x.h declares, with the ctypes table in tinycudann._lib covering
all of them. No compute calls are made here."""
import os
import re
import subprocess

import pytest

from conftest import REPO

HDR = os.path.join(REPO, "include", "tcnn_mi355x.h")
DEBUG_HDR = os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd", "csrc", "debug_api.h")
LIB = os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd", "lib", "libtcnn_mi355x.so")


def header_functions(path=HDR):
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tcnn_[a-z0-9_]+)\s*\(", txt)))


def test_header_parses():
    fns = header_functions()
    assert "tcnn_trainer_training_step" in fns and "tcnn_module_backward" in fns
    assert len(fns) > 40
    # the test-only diagnostics live in the package's debug_api.h, not in the product C-ABI header
    assert not [f for f in fns if f.startswith("tcnn_debug_")]
    assert header_functions(DEBUG_HDR) == ["tcnn_debug_fused_phase_cycles", "tcnn_debug_hfma", "tcnn_debug_peer_loopback", "tcnn_debug_probe"]


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_library_exports_every_declared_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [f for f in header_functions() + header_functions(DEBUG_HDR) if f not in exported]
    assert not missing, missing


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_ctypes_table_covers_header_and_loads():
    from tinycudann import _lib
    assert sorted(_lib.exported_symbols()) == header_functions()
    assert sorted(_lib.debug_symbols()) == header_functions(DEBUG_HDR)
    L = _lib.lib()
    assert L.tcnn_batch_size_granularity() == 256
    assert L.tcnn_default_loss_scale(1) == 128.0 and L.tcnn_default_loss_scale(0) == 1.0
    assert L.tcnn_has_networks() == 1
    assert b"gfx950" in L.tcnn_version()


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_constants_and_enum_orders_match_reference_common_h():
    """The engine's batch granularity, default loss scales and grid enum orders equal the reference's
    include/tiny-cuda-nn/common.h as compiled by oracle/_ref (tests/golden/ref_known_answers.json
    'common_h'): the C-ABI values and the enums of csrc/common.h."""
    import json
    ka = json.load(open(os.path.join(REPO, "tests", "golden", "ref_known_answers.json")))["common_h"]
    from tinycudann import _lib
    L = _lib.lib()
    assert L.tcnn_batch_size_granularity() == ka["batch_size_granularity"]
    assert L.tcnn_default_loss_scale(0) == ka["default_loss_scale_float"]
    txt = open(os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd", "csrc", "common.h")).read()
    for ours, ref in (("GridType", "grid_type"), ("HashType", "hash_type"), ("Interp", "interpolation")):
        body = re.search(r"enum class %s : uint32_t \{([^}]*)\}" % ours, txt).group(1)
        vals = {k.strip(): int(v) for k, v in (e.split("=") for e in body.split(",") if "=" in e)}
        for name, v in vals.items():
            assert ka[ref][name] == v, (ours, name)
