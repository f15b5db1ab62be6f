"""The torch binding's first-order backward fast path (tinycudann/modules.py `_module_function.backward`
without create_graph: one tcnn_module_backward_scaled call) gives the same gradients, bit for bit, as
the reference's differentiable path (modules.py:128-138: doutput * loss_scale, Module::backward,
division by loss_scale -- taken here when create_graph=True), for the parameter and input gradients of
a grid + fused MLP network and of a grid encoding."""
import json
import os

import numpy as np
import pytest

from helpers import CONFIG_HASH

pytestmark = pytest.mark.gpu


def _grads(torch, model, x, create_graph, input_grad=True):
    model.zero_grad(set_to_none=True)
    xi = x.clone().requires_grad_(input_grad)
    out = model(xi)
    loss = ((out.float() - 0.25) ** 2).sum()
    loss.backward(create_graph=create_graph)
    return model.params.grad.detach().clone(), (xi.grad.detach().clone() if input_grad else None)


def test_fused_engine_fast_path_matches_differentiable_path():
    """Without input gradients the network runs the fused engine, whose reductions write the finalised
    fp16(fp16(g) / s) gradient themselves (GradFinalize) -- the same bits as the differentiable path's
    scale / backward / divide sequence."""
    import torch
    import tinycudann as tcnn
    torch.manual_seed(4)
    model = tcnn.NetworkWithInputEncoding(2, 3, CONFIG_HASH["encoding"], CONFIG_HASH["network"]).cuda()
    x = torch.rand(1 << 15, 2, device="cuda")
    gp_fast, _ = _grads(torch, model, x, False, input_grad=False)
    gp_ref, _ = _grads(torch, model, x, True, input_grad=False)
    assert float(gp_fast.abs().max()) > 0
    np.testing.assert_array_equal(gp_fast.cpu().numpy(), gp_ref.cpu().numpy())


@pytest.mark.parametrize("kind", ["network", "grid"])
def test_first_order_fast_path_matches_differentiable_path(kind):
    import torch
    import tinycudann as tcnn
    torch.manual_seed(3)
    if kind == "network":
        model = tcnn.NetworkWithInputEncoding(2, 3, CONFIG_HASH["encoding"], CONFIG_HASH["network"]).cuda()
    else:
        model = tcnn.Encoding(2, CONFIG_HASH["encoding"]).cuda()
    x = torch.rand(4096, 2, device="cuda")
    gp_fast, gx_fast = _grads(torch, model, x, False)
    gp_ref, gx_ref = _grads(torch, model, x, True)
    assert float(gp_fast.abs().max()) > 0 and float(gx_fast.abs().max()) > 0
    np.testing.assert_array_equal(gp_fast.cpu().numpy(), gp_ref.cpu().numpy())
    np.testing.assert_array_equal(gx_fast.cpu().numpy(), gx_ref.cpu().numpy())


@pytest.mark.parametrize("kind", ["network", "grid"])
@pytest.mark.parametrize("create_graph", [False, True])
def test_cpp_autograd_node_matches_python_node(kind, create_graph):
    """The C++ autograd node (csrc/torch_ext.cpp, r06; Module.forward's default once built) and the
    Python autograd.Function it replaces give the same outputs and gradients bit for bit, on the
    first-order fast path and on the differentiable (create_graph) path; for a grid encoding also the
    second-order gradient through Module::backward_backward_input."""
    import torch
    import tinycudann as tcnn
    from tinycudann import modules as M
    assert M._EXT is not None, "the C++ autograd node was not built (neuralbtf-tiny-cuda-nn_amd/build_torch_ext.py)"
    torch.manual_seed(5)
    if kind == "network":
        model = tcnn.NetworkWithInputEncoding(2, 3, CONFIG_HASH["encoding"], CONFIG_HASH["network"]).cuda()
    else:
        model = tcnn.Encoding(2, CONFIG_HASH["encoding"]).cuda()
    x = torch.rand(4096, 2, device="cuda")
    res = {}
    for use_ext in (True, False):
        saved, M._EXT = M._EXT, (M._EXT if use_ext else None)
        try:
            model.zero_grad(set_to_none=True)
            xi = x.clone().requires_grad_(True)
            out = model(xi)
            loss = ((out.float() - 0.25) ** 2).sum()
            loss.backward(create_graph=create_graph)
            r = [out.detach().clone(), model.params.grad.detach().clone(), xi.grad.detach().clone()]
            if create_graph and kind == "grid":
                model.zero_grad(set_to_none=True)
                xj = x.clone().requires_grad_(True)
                o2 = model(xj)
                (gx,) = torch.autograd.grad((o2.float() ** 2).sum(), xj, create_graph=True)
                (gx.square().sum()).backward()
                r.append(model.params.grad.detach().clone())
            res[use_ext] = r
        finally:
            M._EXT = saved
    for a, b in zip(res[True], res[False]):
        np.testing.assert_array_equal(a.float().cpu().numpy(), b.float().cpu().numpy())
