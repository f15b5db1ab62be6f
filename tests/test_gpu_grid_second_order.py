"""GPU parity of the grid's second-order gradients (backward_backward_input,
reference grid.h:351-627 kernels + 902-1026 host, cpp_api.h:94, bindings.cpp:185-239,
modules.py:128-170), through the C-ABI and through torch double-backward, against the oracle
(orc_grid_bwd_bwd, itself pinned to float64 derivatives in test_oracle.py).

Tolerances: dL/dx and dL/d(dL/dy) -- the kernel regroups the reference's per-edge sums per corner
(fp32), rtol 1e-4 of the largest entry; dL/dgrid -- fp32 atomics in any order, then fp16, relative
L2 <= 2e-3 (the reference itself accumulates it with fp16 atomics).
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


def _vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


@pytest.mark.parametrize("interp,D", [("Linear", 2), ("Smoothstep", 2), ("Smoothstep", 3), ("Nearest", 2)])
def test_grid_bwd_bwd_cabi(torch_mod, interp, D):
    torch = torch_mod
    from tinycudann import _lib as L
    lib = L.lib()
    enc = dict(CONFIG_HASH["encoding"], interpolation=interp)
    m = L.check_ptr(lib.tcnn_create_encoding(D, json.dumps(enc).encode(), 1))
    n = lib.tcnn_module_n_params(m)
    W = lib.tcnn_module_n_output_dims(m)
    rng = np.random.default_rng(17 + D)
    table = O.f2h(rng.uniform(-1, 1, n).astype(np.float32))
    p16 = torch.from_numpy(table.view(np.float16)).cuda()
    B = 1024
    pos = rng.uniform(0, 1, (B, D)).astype(np.float32)
    pos_d = torch.from_numpy(pos).cuda()
    out = torch.empty(B, W, dtype=torch.float16, device="cuda")
    ctx = L.check_ptr(lib.tcnn_module_forward(m, None, B, _vp(pos_d), _vp(out), _vp(p16), 1))
    dy = O.f2h(rng.standard_normal((B, W)).astype(np.float32))
    dy_d = torch.from_numpy(dy.view(np.float16)).cuda()
    gx = (rng.standard_normal((B, D)) * 1e-3).astype(np.float32)  # keeps dL/dgrid (~ scale * gx * dy) inside fp16
    gx_d = torch.from_numpy(gx).cuda()
    grad = torch.empty(n, dtype=torch.float16, device="cuda")
    ddy = torch.full((B, W), 7.0, dtype=torch.float16, device="cuda")  # padding columns must come back 0
    dx = torch.empty(B, D, dtype=torch.float32, device="cuda")
    L.check(lib.tcnn_module_backward_backward_input(m, None, ctx, B, _vp(gx_d), _vp(pos_d), _vp(dy_d), _vp(grad), _vp(ddy),
                                                    _vp(dx), _vp(p16)))
    torch.cuda.synchronize()
    g = O.grid_cfg(enc, D)
    LF = g.n_levels * g.n_features_per_level
    rgrad, rddy, rdx = O.grid_bwd_bwd(g, pos, table, gx, np.ascontiguousarray(dy[:, :LF].T))
    got_ddy = ddy.float().cpu().numpy()
    assert np.all(got_ddy[:, LF:] == 0)
    if interp == "Nearest":
        assert np.all(got_ddy == 0) and np.all(dx.cpu().numpy() == 0) and np.all(grad.float().cpu().numpy() == 0)
    else:
        np.testing.assert_allclose(got_ddy[:, :LF], O.h2f(O.f2h(rddy)), rtol=2e-3, atol=1e-4 * np.abs(rddy).max())
        np.testing.assert_allclose(dx.cpu().numpy(), rdx, rtol=1e-4, atol=1e-4 * np.abs(rdx).max())
        assert rel_err(grad.float().cpu().numpy(), rgrad) <= 2e-3
    # dL_ddLdoutput only (no dL/dy, no params): the reference's bindings pass dL_doutput = NULL
    ddy2 = torch.zeros(B, W, dtype=torch.float16, device="cuda")
    L.check(lib.tcnn_module_backward_backward_input(m, None, ctx, B, _vp(gx_d), _vp(pos_d), None, None, _vp(ddy2), None, _vp(p16)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ddy2.cpu().numpy(), ddy.cpu().numpy())
    lib.tcnn_context_destroy(ctx)
    lib.tcnn_module_destroy(m)


def test_encoding_double_backward_autograd(torch_mod):
    """The NeuralBTF / eikonal pattern: gx = d(y.w)/dx with create_graph, then d(gx.v)/d(params, x, w)."""
    torch = torch_mod
    import tinycudann as tcnn
    enc_cfg = dict(CONFIG_HASH["encoding"], interpolation="Smoothstep")
    enc = tcnn.Encoding(2, enc_cfg)
    with torch.no_grad():
        enc.params.uniform_(-1, 1)
    B = 512
    rng = np.random.default_rng(5)
    pos = rng.uniform(0, 1, (B, 2)).astype(np.float32)
    x = torch.from_numpy(pos).cuda().requires_grad_(True)
    w = torch.from_numpy((rng.standard_normal((B, enc.n_output_dims)) * 0.1).astype(np.float16)).cuda().requires_grad_(True)
    v = torch.from_numpy((rng.standard_normal((B, 2)) * 1e-3).astype(np.float32)).cuda()
    y = enc(x)
    L1 = (y * w).float().sum()
    gx = torch.autograd.grad(L1, x, create_graph=True)[0]
    L2 = (gx * v).sum()
    L2.backward()
    torch.cuda.synchronize()
    g = O.grid_cfg(enc_cfg, 2)
    table = enc.params.detach().half().cpu().numpy().view(np.uint16)
    # the first backward receives dL1/dy = w (fp16), scaled by the loss scale 128 (modules.py:126-129)
    dy16 = O.f2h(O.h2f(w.detach().cpu().numpy().view(np.uint16)) * 128.0)
    rgrad, rddy, rdx = O.grid_bwd_bwd(g, pos, table, v.cpu().numpy(), np.ascontiguousarray(dy16.T))
    # first-order result matches too
    np.testing.assert_allclose(gx.detach().cpu().numpy(), O.grid_bwd_input(g, pos, table, np.ascontiguousarray(dy16.T)) / 128.0,
                               rtol=1e-4, atol=1e-4 * np.abs(gx.detach().cpu().numpy()).max())
    np.testing.assert_allclose(x.grad.cpu().numpy(), rdx / 128.0, rtol=1e-4, atol=1e-4 * np.abs(rdx / 128.0).max())
    np.testing.assert_allclose(w.grad.float().cpu().numpy(), O.h2f(O.f2h(rddy)), rtol=2e-3, atol=1e-4 * np.abs(rddy).max())
    assert rel_err(enc.params.grad.cpu().numpy(), rgrad / 128.0) <= 2e-3


def test_network_double_backward_not_implemented(torch_mod):
    """NetworkWithInputEncoding has no backward_backward_input in the reference (object.h:278-288)."""
    torch = torch_mod
    import tinycudann as tcnn
    from tinycudann import _lib as L
    model = tcnn.NetworkWithInputEncoding(2, 3, CONFIG_HASH["encoding"], CONFIG_HASH["network"])
    x = torch.rand(256, 2, device="cuda", requires_grad=True)
    y = model(x)
    gx = torch.autograd.grad(y.float().sum(), x, create_graph=True)[0]
    # a RuntimeError, as the reference's C++ exception through pybind11 (TcnnError, the ctypes path's, is one)
    with pytest.raises(RuntimeError, match="not implemented"):
        gx.sum().backward()
