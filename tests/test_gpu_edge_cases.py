"""Edge cases of the boundary: empty batches, batch granularity errors, wrong
parameter counts -- the calls must fail loudly with tcnn_last_error() or be no-ops, never fault."""
import ctypes
import json

import numpy as np
import pytest

from helpers import CONFIG_HASH, CONFIG_ONEBLOB

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available()
    return torch


def _vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


@pytest.mark.parametrize("cfg", [CONFIG_HASH, CONFIG_ONEBLOB], ids=["hash", "oneblob"])
def test_empty_batch_is_a_noop(torch_mod, cfg):
    torch = torch_mod
    from tinycudann import _lib as L
    lib = L.lib()
    m = L.check_ptr(lib.tcnn_create_network_with_input_encoding(2, 3, json.dumps(cfg["encoding"]).encode(),
                                                                 json.dumps(cfg["network"]).encode()))
    n = lib.tcnn_module_n_params(m)
    p = torch.zeros(n, dtype=torch.float16, device="cuda")
    x = torch.zeros(1, 2, device="cuda")
    out = torch.zeros(1, 16, dtype=torch.float16, device="cuda")
    L.check(lib.tcnn_module_inference(m, None, 0, _vp(x), _vp(out), _vp(p)))
    ctx = L.check_ptr(lib.tcnn_module_forward(m, None, 0, _vp(x), _vp(out), _vp(p), 1))
    g = torch.zeros(n, dtype=torch.float16, device="cuda")
    dx = torch.zeros(1, 2, device="cuda")
    L.check(lib.tcnn_module_backward(m, None, ctx, 0, _vp(dx), _vp(out), _vp(g), _vp(x), _vp(out), _vp(p)))
    torch.cuda.synchronize()
    lib.tcnn_context_destroy(ctx)
    lib.tcnn_module_destroy(m)


def test_batch_granularity_and_bad_config_fail_loudly(torch_mod):
    torch = torch_mod
    from tinycudann import Trainer
    from tinycudann import _lib as L
    lib = L.lib()
    t = Trainer(2, 3, CONFIG_HASH)
    x = torch.rand(100, 2, device="cuda")
    y = torch.rand(100, 3, device="cuda")
    with pytest.raises(L.TcnnError, match="multiple of 256"):
        t.training_step(x, y)
    bad = dict(CONFIG_HASH, network=dict(CONFIG_HASH["network"], n_neurons=48))  # FullyFusedMLP widths
    with pytest.raises(L.TcnnError, match="FullyFusedMLP only supports"):
        Trainer(2, 3, bad)
    assert not lib.tcnn_create_encoding(2, json.dumps({"otype": "Frequency"}).encode(), 1)
    assert "not implemented" in lib.tcnn_last_error().decode()
    # the trainer still works after the failed calls
    x = torch.rand(256, 2, device="cuda")
    y = torch.rand(256, 3, device="cuda")
    t.training_step(x, y)
    assert np.isfinite(t.loss())
