"""GPU parity of the grid options outside the fused engine:
  * stochastic_interpolation (reference grid.h:284-298, random_val common_device.h:333-337): the
    backward sends each (point, level) gradient to one corner picked by pcg32{1337}.advance(i + l*B);
  * max_level masking, scalar and per point (grid_interface.h:101-123; grid.h:69-91 forward,
    236-244 backward, 376-384 / 482-490 second order).
Both run on the layer-wise engine (the fused kernel does not take them; the trainer switches engine
per step). Tolerances: forward bit-exact; grid gradients (int32 fixed-point sums) relative L2 <= 1e-3;
trainer gradients as the other layered tests (2e-3).
"""
import copy
import ctypes
import json

import numpy as np
import pytest

from helpers import CONFIG_HASH, make_batch, rel_err, trainer_arrays
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available()
    return torch


def _vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _grid_module(lib, L, enc):
    return L.check_ptr(lib.tcnn_create_encoding(2, json.dumps(enc).encode(), 1))


def _run_module(torch, lib, L, m, table, pos, dy):
    B = pos.shape[0]
    W = lib.tcnn_module_n_output_dims(m)
    n = lib.tcnn_module_n_params(m)
    p16 = torch.from_numpy(table.view(np.float16)).cuda()
    pos_d = torch.from_numpy(pos).cuda()
    out = torch.empty(B, W, dtype=torch.float16, device="cuda")
    ctx = L.check_ptr(lib.tcnn_module_forward(m, None, B, _vp(pos_d), _vp(out), _vp(p16), 1))
    dy_d = torch.from_numpy(dy.view(np.float16)).cuda()
    grad = torch.empty(n, dtype=torch.float16, device="cuda")
    dx = torch.empty(B, 2, dtype=torch.float32, device="cuda")
    L.check(lib.tcnn_module_backward(m, None, ctx, B, _vp(dx), _vp(dy_d), _vp(grad), _vp(pos_d), _vp(out), _vp(p16)))
    torch.cuda.synchronize()
    lib.tcnn_context_destroy(ctx)
    return out.cpu().numpy().view(np.uint16), grad.float().cpu().numpy(), dx.cpu().numpy()


def test_stochastic_interpolation_backward(torch_mod):
    torch = torch_mod
    from tinycudann import _lib as L
    lib = L.lib()
    enc = dict(CONFIG_HASH["encoding"], stochastic_interpolation=True)
    m = _grid_module(lib, L, enc)
    g = O.grid_cfg(enc, 2)
    rng = np.random.default_rng(12)
    table = O.f2h(rng.uniform(-1, 1, g.n_params).astype(np.float32))
    B = 4096
    pos = rng.uniform(0, 1, (B, 2)).astype(np.float32)
    W = lib.tcnn_module_n_output_dims(m)
    dy = O.f2h(rng.standard_normal((B, W)).astype(np.float32))
    out, grad, dx = _run_module(torch, lib, L, m, table, pos, dy)
    LF = g.n_levels * g.n_features_per_level
    np.testing.assert_array_equal(out.T[:LF], O.grid_fwd(g, pos, table))  # forward unaffected
    ref = O.grid_bwd(g, pos, np.ascontiguousarray(dy[:, :LF].T))
    assert rel_err(grad, ref) <= 1e-3
    g_lin = O.grid_cfg(dict(CONFIG_HASH["encoding"]), 2)
    assert rel_err(grad, O.grid_bwd(g_lin, pos, np.ascontiguousarray(dy[:, :LF].T))) > 0.1  # really stochastic
    lib.tcnn_module_destroy(m)


@pytest.mark.parametrize("per_point", [False, True])
def test_max_level_masking(torch_mod, per_point):
    torch = torch_mod
    from tinycudann import _lib as L
    lib = L.lib()
    enc = dict(CONFIG_HASH["encoding"])
    m = _grid_module(lib, L, enc)
    g = O.grid_cfg(enc, 2)
    rng = np.random.default_rng(13)
    table = O.f2h(rng.uniform(-1, 1, g.n_params).astype(np.float32))
    B = 2048
    pos = rng.uniform(0, 1, (B, 2)).astype(np.float32)
    if per_point:
        ml = rng.uniform(0, 1, B).astype(np.float32)
        ml_d = torch.from_numpy(ml).cuda()
        L.check(lib.tcnn_module_set_max_level_gpu(m, _vp(ml_d)))
        O.grid_set_max_level(g, 0.0, ml)
    else:
        L.check(lib.tcnn_module_set_max_level(m, 0.45))
        assert abs(lib.tcnn_module_max_level(m) - 0.45) < 1e-7
        O.grid_set_max_level(g, 0.45)
    W = lib.tcnn_module_n_output_dims(m)
    dy = O.f2h(rng.standard_normal((B, W)).astype(np.float32))
    out, grad, dx = _run_module(torch, lib, L, m, table, pos, dy)
    LF = g.n_levels * g.n_features_per_level
    ref_out = O.grid_fwd(g, pos, table)
    np.testing.assert_array_equal(out.T[:LF], ref_out)
    assert np.any(ref_out == 0)
    dyT = np.ascontiguousarray(dy[:, :LF].T)
    assert rel_err(grad, O.grid_bwd(g, pos, dyT)) <= 1e-3
    np.testing.assert_allclose(dx, O.grid_bwd_input(g, pos, table, dyT), rtol=1e-5, atol=1e-5)
    lib.tcnn_module_destroy(m)


def test_trainer_stochastic_interpolation_step(torch_mod):
    torch = torch_mod
    from tinycudann import Trainer
    cfg = copy.deepcopy(CONFIG_HASH)
    cfg["encoding"]["stochastic_interpolation"] = True
    t = Trainer(2, 3, cfg, seed=1337)
    assert t.engine == "fused", t.engine  # the tile engine (the register-resident kernel takes no grid options)
    om = O.OracleModel(cfg, 2, 3, seed=1337)
    B = 1024
    pos, tgt = make_batch(B)
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    loss_ref = om.train_step(pos, tgt, run_optimizer=False, n_threads=4)
    assert abs(t.loss() - loss_ref) <= 1e-3 * abs(loss_ref)
    a = trainer_arrays(t)
    nm = om.n_mlp_params
    assert rel_err(a["g32"][:nm], om.grad32[:nm]) <= 2e-3
    assert rel_err(a["g32"][nm:], om.grad32[nm:]) <= 2e-3


def test_trainer_max_level_switches_engine(torch_mod):
    torch = torch_mod
    from tinycudann import Trainer
    from tinycudann import _lib as L
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    assert t.engine == "fused"
    L.check(L.lib().tcnn_trainer_set_max_level(t.h, 0.5))
    assert t.engine == "fused"  # now the tile engine: encoding pass + grid backward take the mask
    B = 1024
    pos, tgt = make_batch(B)
    for _ in range(3):
        t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda())
    l1 = t.loss()
    a = trainer_arrays(t)
    nm = t.n_network_params
    gg = a["g32"][nm:]
    g = O.grid_cfg(CONFIG_HASH["encoding"], 2)
    assert np.all(gg[g.offsets[9] * 2:] == 0)  # masked levels get no gradient
    L.check(L.lib().tcnn_trainer_set_max_level(t.h, 1000.0))
    assert t.engine == "fused"
    for _ in range(3):
        t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda())
    assert np.isfinite(l1) and np.isfinite(t.loss())
