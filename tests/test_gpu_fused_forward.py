"""The one-kernel grid + MLP forward (k_fused_fwd_grid: inference and the forward of a training context)
against the two-pass forward it replaces (the SoA grid forward, then k_mlp_infer; TCNN_SPLIT_FORWARD,
read when a module is built): outputs, and the gradients of a backward that reads the kept encoding,
bit for bit -- positions inside [0, 1] (the branch-free index) and outside (the general index), 2-D and
3-D grids. Reference: the encoding's forward (grid.h:48-212) feeding kernel_mlp_fused<...,
INFERENCE=true> (fully_fused_mlp.cu:499-557); both paths are pinned to the oracle by
tests/test_gpu_parity.py and test_gpu_module_context.py."""
import os

import numpy as np
import pytest

from helpers import CONFIG_HASH

pytestmark = pytest.mark.gpu


def _pair(tcnn, n_in):
    a = tcnn.NetworkWithInputEncoding(n_in, 3, CONFIG_HASH["encoding"], CONFIG_HASH["network"]).cuda()
    os.environ["TCNN_SPLIT_FORWARD"] = "1"
    try:
        b = tcnn.NetworkWithInputEncoding(n_in, 3, CONFIG_HASH["encoding"], CONFIG_HASH["network"]).cuda()
    finally:
        del os.environ["TCNN_SPLIT_FORWARD"]
    with __import__("torch").no_grad():
        b.params.copy_(a.params)
    return a, b


@pytest.mark.parametrize("n_in", [2, 3])
@pytest.mark.parametrize("span", ["inside", "outside"])
def test_fused_forward_matches_two_pass_forward(n_in, span):
    import torch
    import tinycudann as tcnn
    torch.manual_seed(11)
    a, b = _pair(tcnn, n_in)
    x = torch.rand(1 << 16, n_in, device="cuda")
    if span == "outside":
        x = x * 1.4 - 0.2  # some positions outside [0, 1]: the general index path
    with torch.no_grad():
        ya, yb = a(x), b(x)
    assert torch.isfinite(ya).all() and float(ya.abs().max()) > 0
    np.testing.assert_array_equal(ya.cpu().numpy(), yb.cpu().numpy())
    # training context: the forward keeps its encoding, the backward reads it
    grads = []
    for m in (a, b):
        m.zero_grad(set_to_none=True)
        y = m(x)
        ((y.float() - 0.3) ** 2).mean().backward()
        grads.append((y.detach().cpu().numpy(), m.params.grad.detach().cpu().numpy()))
    np.testing.assert_array_equal(grads[0][0], grads[1][0])
    assert np.abs(grads[0][1]).max() > 0
    np.testing.assert_array_equal(grads[0][1], grads[1][1])


def test_trainer_inference_matches_two_pass_forward():
    import torch
    from tinycudann import Trainer
    torch.manual_seed(5)
    x = torch.rand(1 << 15, 2, device="cuda")
    t = torch.rand(1 << 15, 3, device="cuda")
    ta = Trainer(2, 3, CONFIG_HASH, seed=1337)
    os.environ["TCNN_SPLIT_FORWARD"] = "1"
    try:
        tb = Trainer(2, 3, CONFIG_HASH, seed=1337)
    finally:
        del os.environ["TCNN_SPLIT_FORWARD"]
    for _ in range(3):
        ta.training_step(x, t)
        tb.training_step(x, t)
    ya, yb = ta.inference(x), tb.inference(x)
    assert float(ya.abs().max()) > 0
    np.testing.assert_array_equal(ya.cpu().numpy(), yb.cpu().numpy())


def test_unaligned_parameter_view():
    """A parameter tensor that is a view at an 8-byte offset into a flat fp16 buffer (not 16-byte aligned:
    the in-kernel LDS image build uses 16-byte loads) runs through the packed weight image instead of
    failing: inference and the kept-context backward bit-identical to the aligned tensor."""
    import ctypes
    import torch
    from tinycudann import _lib as L
    lib = L.lib()
    import json
    m = L.check_ptr(lib.tcnn_create_network_with_input_encoding(2, 3, json.dumps(CONFIG_HASH["encoding"]).encode(),
                                                                 json.dumps(CONFIG_HASH["network"]).encode()))
    n = lib.tcnn_module_n_params(m)
    p32 = torch.zeros(n, dtype=torch.float32, device="cuda")
    L.check(lib.tcnn_module_initialize_params(m, 1337, ctypes.c_void_p(p32.data_ptr()), 1.0))
    aligned = p32.half().contiguous()
    flat = torch.zeros(n + 8, dtype=torch.float16, device="cuda")
    view = flat[4:4 + n]
    view.copy_(aligned)
    assert view.data_ptr() % 16 == 8
    B = 4096
    x = torch.rand(B, 2, device="cuda")
    outs = []
    for p in (aligned, view):
        out = torch.empty(B, 16, dtype=torch.float16, device="cuda")
        L.check(lib.tcnn_module_inference(m, None, B, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                          ctypes.c_void_p(p.data_ptr())))
        ctx = L.check_ptr(lib.tcnn_module_forward(m, None, B, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                                  ctypes.c_void_p(p.data_ptr()), 0))
        dout = torch.full((B, 16), 0.01, dtype=torch.float16, device="cuda")
        grad = torch.empty(n, dtype=torch.float16, device="cuda")
        L.check(lib.tcnn_module_backward(m, None, ctx, B, None, ctypes.c_void_p(dout.data_ptr()), ctypes.c_void_p(grad.data_ptr()),
                                         ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(p.data_ptr())))
        torch.cuda.synchronize()
        lib.tcnn_context_destroy(ctx)
        outs.append((out.cpu().numpy(), grad.cpu().numpy()))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    lib.tcnn_module_destroy(m)
