"""GPU tests of Trainer::forward / backward (reference include/tiny-cuda-nn/trainer.h:97-153) and the
training_step options they carry (trainer.h:163-203): data_pdf, external dL/dy, dL/dinput and
Accumulate gradients.

  * forward + backward + optimizer_step reproduce training_step bit for bit on the three engines
    (the register-resident fused kernel, the tile kernel, the layer-wise engine): same dL/dy (the
    standalone loss kernel rounds exactly like the fused one), same gradient summation orders
  * data_pdf (relative_l2.h:64-72): the loss and gradient divide by the pdf -- pdf = 2 halves them
    exactly (a division by 2 is exact and commutes with the fp16 rounding above the subnormals); a
    random pdf gives the numpy loss of the context's own output within fp32 summation error
  * external dL/dy: the context's own dL/doutput fed back as external_dL_dy gives the same gradients
  * Accumulate: two backward passes give twice the Overwrite gradient (exact in fp32)
  * dL/dinput: equal to the runtime Module's dL/dinput for the same parameters and dL/dy
"""
import copy
import ctypes

import numpy as np
import pytest

from helpers import CONFIG_HASH, CONFIG_ONEBLOB, make_batch, trainer_arrays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available()
    return torch


def _cfg(which):
    if which == "fused":
        return copy.deepcopy(CONFIG_HASH)
    cfg = copy.deepcopy(CONFIG_ONEBLOB)
    cfg["network"] = dict(cfg["network"], n_neurons=64, n_hidden_layers=2)
    if which == "layered":
        cfg["network"]["otype"] = "CutlassMLP"
    return cfg


def _batch(torch, B, step=0):
    pos, tgt = make_batch(B, step=step)
    return torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda()


@pytest.mark.parametrize("which", ["fused", "tile", "layered"])
def test_forward_backward_optimizer_equals_training_step(torch_mod, which):
    torch = torch_mod
    from tinycudann import Trainer
    cfg = _cfg(which)
    a, b = Trainer(2, 3, cfg, seed=1337), Trainer(2, 3, cfg, seed=1337)
    assert a.engine == ("layered" if which == "layered" else "fused")
    B = 4096
    for s in range(3):
        x, y = _batch(torch, B, s)
        a.training_step(x, y)
        ctx = b.forward(x, y)
        b.backward(ctx, x)
        b.optimizer_step()
        la, lb = a.loss(), ctx.loss()
        assert abs(la - lb) <= 1e-6 * abs(la), (s, la, lb)  # loss sums differ only in summation order
    ra, rb = trainer_arrays(a), trainer_arrays(b)
    np.testing.assert_array_equal(ra["w16"], rb["w16"])
    np.testing.assert_array_equal(ra["w32"], rb["w32"])


def test_data_pdf_scales_loss_and_gradients(torch_mod):
    torch = torch_mod
    from tinycudann import Trainer
    cfg = _cfg("fused")
    B = 4096
    x, y = _batch(torch, B)
    t = Trainer(2, 3, cfg, seed=1337)
    c1 = t.forward(x, y)
    t.backward(c1, x)
    g1, l1 = trainer_arrays(t)["g32"], c1.loss()
    d1 = c1.dL_doutput.cpu().numpy().astype(np.float32)
    two = torch.full((B, 3), 2.0, device="cuda")
    c2 = t.forward(x, y, data_pdf=two)
    t.backward(c2, x)
    g2, l2 = trainer_arrays(t)["g32"], c2.loss()
    d2 = c2.dL_doutput.cpu().numpy().astype(np.float32)
    assert l2 == pytest.approx(l1 / 2, rel=1e-6)
    normal = np.abs(d1) >= 2.0 ** -13  # halving stays above the fp16 subnormals: exact
    np.testing.assert_array_equal(d2[normal], d1[normal] / 2)
    np.testing.assert_allclose(g2, g1 / 2, rtol=1e-3, atol=1e-6 * np.abs(g1).max())
    # a random pdf: the loss against numpy on the context's own output
    rng = np.random.default_rng(7)
    pdf = rng.uniform(0.25, 4.0, size=(B, 3)).astype(np.float32)
    c3 = t.forward(x, y, data_pdf=torch.from_numpy(pdf).cuda())
    p = c3.output.cpu().numpy().astype(np.float64)[:, :3]
    tg = y.cpu().numpy().astype(np.float64)
    ref = ((p - tg) ** 2 / (p * p + 0.01) / pdf / (B * 3)).sum()
    assert c3.loss() == pytest.approx(ref, rel=1e-5)


@pytest.mark.parametrize("which", ["fused", "tile", "layered"])
def test_external_dL_dy_and_accumulate(torch_mod, which):
    torch = torch_mod
    from tinycudann import Trainer
    t = Trainer(2, 3, _cfg(which), seed=1337)
    B = 4096
    x, y = _batch(torch, B)
    c = t.forward(x, y)
    t.backward(c, x)
    g_loss = trainer_arrays(t)["g32"]
    dy = c.dL_doutput.contiguous()
    assert dy.shape == (B, t.padded_output_width)
    ce = t.forward(x, external_dL_dy=dy)
    assert ce.loss() == 0.0
    t.backward(ce, x)
    np.testing.assert_array_equal(trainer_arrays(t)["g32"], g_loss)
    t.backward(ce, x, accumulate=True)
    np.testing.assert_array_equal(trainer_arrays(t)["g32"], 2 * g_loss)
    # GradientMode::Ignore (common.h, trainer.h:146-153): parameter gradients untouched, dL/dinput written
    ci = t.forward(x, y, prepare_input_gradients=True)
    dx = torch.zeros(B, 2, device="cuda")
    t.backward(ci, x, dL_dinput=dx, gradient_mode="ignore")
    np.testing.assert_array_equal(trainer_arrays(t)["g32"], 2 * g_loss)
    dx2 = torch.zeros(B, 2, device="cuda")
    t.backward(ci, x, dL_dinput=dx2)
    np.testing.assert_array_equal(dx.cpu().numpy(), dx2.cpu().numpy())
    assert float(dx.abs().max()) > 0


@pytest.mark.parametrize("which", ["fused", "tile"])
def test_dL_dinput_matches_module(torch_mod, which):
    torch = torch_mod
    from tinycudann import Trainer, _lib as L
    import json
    cfg = _cfg(which)
    t = Trainer(2, 3, cfg, seed=1337)
    B = 2048
    x, y = _batch(torch, B)
    c = t.forward(x, y, prepare_input_gradients=True)
    dx = torch.zeros(B, 2, device="cuda")
    t.backward(c, x, dL_dinput=dx)
    dy = c.dL_doutput.contiguous()
    # the runtime Module on the trainer's fp16 parameters, same dL/dy
    lib = L.lib()
    m = L.check_ptr(lib.tcnn_create_network_with_input_encoding(2, 3, json.dumps(cfg["encoding"]).encode(),
                                                                json.dumps(cfg["network"]).encode()))
    params = ctypes.c_void_p(lib.tcnn_trainer_params(t.h))
    out = torch.empty(B, t.padded_output_width, dtype=torch.float16, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    mc = L.check_ptr(lib.tcnn_module_forward(m, s, B, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()), params, 1))
    dx_m = torch.zeros(B, 2, device="cuda")
    L.check(lib.tcnn_module_backward(m, s, mc, B, ctypes.c_void_p(dx_m.data_ptr()), ctypes.c_void_p(dy.data_ptr()), None,
                                     ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()), params))
    torch.cuda.synchronize()
    lib.tcnn_context_destroy(mc)
    lib.tcnn_module_destroy(m)
    assert float(dx.abs().max()) > 0
    np.testing.assert_array_equal(dx.cpu().numpy(), dx_m.cpu().numpy())
