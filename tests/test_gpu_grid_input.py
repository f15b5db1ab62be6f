"""GPU parity of dL/dinput through the multiresolution grid (reference kernel_grid's
dy_dx branch grid.h:171-211 + kernel_grid_backward_input grid.h:322-349), which this engine fuses
into one kernel that recomputes dy/dx from the table.

Tolerances: grid module alone -- same fp32 operation order as the oracle, rtol 1e-5; network +
grid -- dL/d(encoding) passes through fp16 like the reference's, relative L2 <= 2e-3.
"""
import ctypes
import json

import numpy as np
import pytest

from helpers import CONFIG_HASH, make_batch, rel_err
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available()
    return torch


@pytest.mark.parametrize("interp", ["Linear", "Smoothstep"])
def test_grid_module_input_gradient(torch_mod, interp):
    torch = torch_mod
    from tinycudann import _lib as L
    lib = L.lib()
    enc = dict(CONFIG_HASH["encoding"], interpolation=interp)
    m = L.check_ptr(lib.tcnn_create_encoding(2, json.dumps(enc).encode(), 1))
    n = lib.tcnn_module_n_params(m)
    W = lib.tcnn_module_n_output_dims(m)
    rng = np.random.default_rng(9)
    table = O.f2h(rng.uniform(-1, 1, n).astype(np.float32))
    p16 = torch.from_numpy(table.view(np.float16)).cuda()
    B = 1024
    pos, _ = make_batch(B, seed=21)
    pos_d = torch.from_numpy(pos).cuda()
    out = torch.empty(B, W, dtype=torch.float16, device="cuda")
    ctx = L.check_ptr(lib.tcnn_module_forward(m, None, B, ctypes.c_void_p(pos_d.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                              ctypes.c_void_p(p16.data_ptr()), 1))
    dy = O.f2h(rng.standard_normal((B, W)).astype(np.float32))
    dy_d = torch.from_numpy(dy.view(np.float16)).cuda()
    dx = torch.empty(B, 2, dtype=torch.float32, device="cuda")
    grad = torch.empty(n, dtype=torch.float16, device="cuda")
    L.check(lib.tcnn_module_backward(m, None, ctx, B, ctypes.c_void_p(dx.data_ptr()), ctypes.c_void_p(dy_d.data_ptr()),
                                     ctypes.c_void_p(grad.data_ptr()), ctypes.c_void_p(pos_d.data_ptr()),
                                     ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(p16.data_ptr())))
    torch.cuda.synchronize()
    g = O.grid_cfg(enc, 2)
    ref = O.grid_bwd_input(g, pos, table, np.ascontiguousarray(dy.T))
    np.testing.assert_allclose(dx.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    # parameter gradient of the same call (bit-reproducible fixed-point sums vs fp32 oracle)
    gref = O.grid_bwd(g, pos, np.ascontiguousarray(dy.T))
    assert rel_err(grad.float().cpu().numpy(), gref) <= 1e-3
    lib.tcnn_context_destroy(ctx)
    lib.tcnn_module_destroy(m)


def test_network_with_grid_input_gradient(torch_mod):
    torch = torch_mod
    from tinycudann import _lib as L
    lib = L.lib()
    enc, net = CONFIG_HASH["encoding"], CONFIG_HASH["network"]
    m = L.check_ptr(lib.tcnn_create_network_with_input_encoding(2, 3, json.dumps(enc).encode(), json.dumps(net).encode()))
    n = lib.tcnn_module_n_params(m)
    p32 = torch.zeros(n, dtype=torch.float32, device="cuda")
    L.check(lib.tcnn_module_initialize_params(m, 7, ctypes.c_void_p(p32.data_ptr()), 1.0))
    p32[O.mlp_n_params(64, 32, 2, 16):] *= 5000.0  # O(1) grid values so dy/dx is exercised
    p16 = p32.half().contiguous()
    B = 512
    pos, _ = make_batch(B, seed=5)
    pos_d = torch.from_numpy(pos).cuda()
    out = torch.empty(B, 16, dtype=torch.float16, device="cuda")
    ctx = L.check_ptr(lib.tcnn_module_forward(m, None, B, ctypes.c_void_p(pos_d.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                              ctypes.c_void_p(p16.data_ptr()), 1))
    dout = np.zeros((B, 16), np.float32)
    dout[:, :3] = np.random.default_rng(4).standard_normal((B, 3))
    dout16 = torch.from_numpy(dout).half().cuda()
    dx = torch.empty(B, 2, dtype=torch.float32, device="cuda")
    L.check(lib.tcnn_module_backward(m, None, ctx, B, ctypes.c_void_p(dx.data_ptr()), ctypes.c_void_p(dout16.data_ptr()), None,
                                     ctypes.c_void_p(pos_d.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                     ctypes.c_void_p(p16.data_ptr())))
    torch.cuda.synchronize()
    params16 = p16.cpu().numpy().view(np.uint16)
    g = O.grid_cfg(enc, 2)
    nm = O.mlp_n_params(64, 32, 2, 16)
    encv = O.grid_fwd(g, pos, params16[nm:])
    _, hidden = O.mlp_fwd(64, 32, 2, 16, params16[:nm], encv)
    _, denc = O.mlp_bwd(64, 32, 2, 16, params16[:nm], encv, hidden, dout16.cpu().numpy().view(np.uint16))
    ref = O.grid_bwd_input(g, pos, params16[nm:], denc)
    assert rel_err(dx.cpu().numpy(), ref) <= 2e-3, rel_err(dx.cpu().numpy(), ref)
    lib.tcnn_context_destroy(ctx)
    lib.tcnn_module_destroy(m)


def test_torch_autograd_input_gradient(torch_mod):
    """tinycudann.NetworkWithInputEncoding (modules.py mirror): x.requires_grad gives dL/dx through
    the MLP and the hash grid, equal to the Module-level backward (loss scale 128 handled as in the
    reference's autograd function, modules.py:126-129); Encoding and Network (Identity) too."""
    torch = torch_mod
    import tinycudann as tcnn
    torch.manual_seed(0)
    for model in (tcnn.NetworkWithInputEncoding(2, 3, CONFIG_HASH["encoding"], CONFIG_HASH["network"]),
                  tcnn.Encoding(2, CONFIG_HASH["encoding"]),
                  tcnn.Network(2, 3, CONFIG_HASH["network"])):
        if isinstance(model, tcnn.Encoding):
            with torch.no_grad():
                model.params.mul_(1000.0)  # O(0.1) table values
        x = torch.rand(512, 2, device="cuda", requires_grad=True)
        y = model(x)
        y.float().square().sum().backward()
        assert x.grad is not None and torch.isfinite(x.grad).all()
        assert x.grad.abs().sum() > 0
        assert model.params.grad is not None and torch.isfinite(model.params.grad).all()
