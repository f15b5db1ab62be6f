"""GPU parity of the HIP hot path against the CPU oracle (oracle/), seeded inputs, config_hash.json.

Tolerances (north_star: outputs within 1e-3 relative fp16 tolerance):
  * grid encoding forward: bit-exact (same fp16 FMA chain, same index math)
  * network output: |gpu - oracle| <= 2 fp16 ulp (fp32 MFMA vs fp32 CPU summation order)
  * loss sum and gradient vectors: relative L2 error <= 1e-3
  * Adam: bit-exact (masters, fp16 copies, moments, step counts) over 6 steps on the same fp16 gradients
"""
import ctypes
import json

import numpy as np
import pytest

from helpers import (CONFIG_HASH, assert_trainer_grads_per_element, assert_wgrad_per_element, assert_within_fp16_ulps, make_batch,
                     rel_err, relu_margin_ok, relu_safe_grid_batch, trainer_arrays, trainer_grad_bounds)
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_grid_forward_bit_exact(torch_mod):
    torch = torch_mod
    from tinycudann import _lib as L
    lib = L.lib()
    enc = CONFIG_HASH["encoding"]
    m = L.check_ptr(lib.tcnn_create_encoding(2, json.dumps(enc).encode(), 1))
    n = lib.tcnn_module_n_params(m)
    p32 = torch.zeros(n, dtype=torch.float32, device="cuda")
    L.check(lib.tcnn_module_initialize_params(m, 1337, ctypes.c_void_p(p32.data_ptr()), 1.0))
    # widen the init range so interpolation rounding is exercised on O(1) values
    p16 = (p32 * 5000.0).half().contiguous()
    for B in (256, 4096):
        pos, _ = make_batch(B, seed=7)
        pos_d = torch.from_numpy(pos).cuda()
        out = torch.empty(B, lib.tcnn_module_n_output_dims(m), dtype=torch.float16, device="cuda")
        L.check(lib.tcnn_module_inference(m, None, B, ctypes.c_void_p(pos_d.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                          ctypes.c_void_p(p16.data_ptr())))
        torch.cuda.synchronize()
        g = O.grid_cfg(enc, 2)
        ref = O.grid_fwd(g, pos, p16.cpu().numpy().view(np.uint16))  # SoA [32][B]
        got = out.cpu().numpy().view(np.uint16).T
        np.testing.assert_array_equal(got, ref)
    lib.tcnn_module_destroy(m)


def test_trainer_init_matches_oracle(torch_mod):
    from tinycudann import Trainer
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    om = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
    a = trainer_arrays(t)
    np.testing.assert_array_equal(a["w32"], om.w32)
    np.testing.assert_array_equal(a["w16"], om.w16)


@pytest.mark.parametrize("B", [256, 4096])
def test_fused_step_gradients_and_loss(torch_mod, B):
    torch = torch_mod
    from tinycudann import Trainer
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    assert t.engine == "fused"
    om = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
    pos, tgt = make_batch(B)
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    loss_gpu = t.loss()
    loss_ref = om.train_step(pos, tgt, run_optimizer=False)
    assert abs(loss_gpu - loss_ref) <= 1e-3 * abs(loss_ref), (loss_gpu, loss_ref)
    a = trainer_arrays(t)
    nm = om.n_mlp_params
    e_mlp = rel_err(a["g32"][:nm], om.grad32[:nm])
    e_grid = rel_err(a["g32"][nm:], om.grad32[nm:])
    assert e_mlp <= 1e-3, e_mlp
    assert e_grid <= 1e-3, e_grid

    # per element, on a batch clear of the ReLU boundaries (helpers.relu_margin_ok): every term of
    # each sum within 8 fp16 ulps (helpers.trainer_grad_bounds)
    t2 = Trainer(2, 3, CONFIG_HASH, seed=1337)
    om2 = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
    pos, tgt = relu_safe_grid_batch(CONFIG_HASH, om2.w16, B)
    t2.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    om2.train_step(pos, tgt, run_optimizer=False)
    a2 = trainer_arrays(t2)
    mag, gb = trainer_grad_bounds(CONFIG_HASH, a2["w16"], pos, tgt)
    assert_trainer_grads_per_element(a2["g32"], om2.grad32, nm, mag, gb)


def test_fused_step_positions_outside_unit_square(torch_mod):
    """The fused kernel takes a branch-free grid index when every position of a wave's slice is in
    [0, 1] and the general one (with the reference's `% size` wrap, common_device.h:706) otherwise:
    a batch whose second half lies in [-0.5, 1.5] runs both paths, against the oracle."""
    torch = torch_mod
    from tinycudann import Trainer
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    om = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
    B = 4096
    pos, tgt = make_batch(B, seed=5)
    pos[B // 2:] = pos[B // 2:] * 2.0 - 0.5
    pos[B // 2 + 7] = [1.0, 0.0]  # the edges are in range
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    loss_gpu = t.loss()
    loss_ref = om.train_step(pos, tgt, run_optimizer=False)
    assert abs(loss_gpu - loss_ref) <= 1e-3 * abs(loss_ref), (loss_gpu, loss_ref)
    a = trainer_arrays(t)
    nm = om.n_mlp_params
    assert rel_err(a["g32"][:nm], om.grad32[:nm]) <= 1e-3
    assert rel_err(a["g32"][nm:], om.grad32[nm:]) <= 1e-3


def test_adam_step_matches_oracle_on_same_gradients(torch_mod):
    """Adam in isolation, bit for bit: the oracle's Adam is fed the GPU's own fp16 gradients each step
    (network parameters in the grid backward's tail, grid parameters in k_adam); fp32 masters, fp16
    copies, both moments and the per-parameter step counts must be identical after every step --
    including the steps whose bias-correction factor sqrt(1 - b2^t) / (1 - b1^t) a device powf
    rounds differently from the C library's (the engine computes that table on the host)."""
    torch = torch_mod
    from tinycudann import Trainer
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    om = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
    w32, w16 = om.w32.copy(), om.w16.copy()
    m1 = np.zeros(om.n_params, np.float32); m2 = np.zeros_like(m1); steps = np.zeros(om.n_params, np.uint32)
    for s in range(6):
        pos, tgt = make_batch(4096, step=s)
        t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=True)
        a = trainer_arrays(t)
        # the GPU wrote its fp16 gradients (grad32 rounded) into param_gradients before the update
        O.adam_step(om.m.adam, om.n_mlp_params, 128.0, s + 1, w32, w16, a["g16"], m1, m2, steps)
        gm1, gm2, gst = [x.cpu().numpy() for x in t.optimizer_state()]
        for name, got, ref in (("w32", a["w32"], w32), ("w16", a["w16"], w16), ("m1", gm1, m1), ("m2", gm2, m2), ("steps", gst, steps)):
            assert np.array_equal(got.view(np.uint32) if got.dtype == np.float32 else got,
                                  ref.view(np.uint32) if ref.dtype == np.float32 else ref), (s, name, int(np.sum(got != ref)))


@pytest.mark.parametrize("grid_gain", [1.0, 5000.0])
def test_inference_matches_oracle(torch_mod, grid_gain):
    """Trainer inference (grid forward + the fused inference kernel) vs the oracle, at the init
    scale and with the grid parameters scaled to O(1) outputs, on a batch that is not a multiple of
    the inference kernel's 64-sample workgroup."""
    torch = torch_mod
    from tinycudann import Trainer
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    om = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
    if grid_gain != 1.0:
        w = om.w32.copy()
        w[om.n_mlp_params:] *= grid_gain
        t.set_params_full_precision(w)
        om.w32[:] = w
        om.w16[:] = O.f2h(w)
    pos, _ = make_batch(2048 + 96, seed=3)
    out = t.inference(torch.from_numpy(pos).cuda()).cpu().numpy()
    ref = O.h2f(om.inference(pos))[:, :3]
    assert_within_fp16_ulps(out, ref)


def test_training_trajectory_tracks_oracle(torch_mod):
    torch = torch_mod
    from tinycudann import Trainer
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    om = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
    B = 2048
    lg, lr = [], []
    for s in range(12):
        pos, tgt = make_batch(B, step=s)
        t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda())
        lg.append(t.loss())
        lr.append(om.train_step(pos, tgt, n_threads=4))
    lg, lr = np.array(lg), np.array(lr)
    assert lg[-1] < 0.5 * lg[0]
    np.testing.assert_allclose(lg, lr, rtol=3e-2)


def test_module_backward_matches_oracle(torch_mod):
    """cpp_api Module::backward with an external dL/doutput (Overwrite) vs oracle."""
    torch = torch_mod
    from tinycudann import _lib as L
    lib = L.lib()
    enc, net = CONFIG_HASH["encoding"], CONFIG_HASH["network"]
    m = L.check_ptr(lib.tcnn_create_network_with_input_encoding(2, 3, json.dumps(enc).encode(), json.dumps(net).encode()))
    n = lib.tcnn_module_n_params(m)
    p32 = torch.zeros(n, dtype=torch.float32, device="cuda")
    L.check(lib.tcnn_module_initialize_params(m, 42, ctypes.c_void_p(p32.data_ptr()), 1.0))
    p16 = p32.half().contiguous()
    B = 1024
    pos, _ = make_batch(4 * B, seed=11)
    # a batch clear of the ReLU boundaries, so the per-element bounds below apply (helpers.relu_margin_ok)
    g0 = O.grid_cfg(enc, 2)
    p0 = p16.cpu().numpy().view(np.uint16)
    nm0 = O.mlp_n_params(64, 32, 2, 16)
    ok = relu_margin_ok(64, 32, 2, p0[:nm0], O.h2f(O.grid_fwd(g0, pos, p0[nm0:])).T)
    pos = np.ascontiguousarray(pos[np.nonzero(ok)[0][:B]])
    assert pos.shape[0] == B
    pos_d = torch.from_numpy(pos).cuda()
    out = torch.empty(B, 16, dtype=torch.float16, device="cuda")
    ctx = L.check_ptr(lib.tcnn_module_forward(m, None, B, ctypes.c_void_p(pos_d.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                              ctypes.c_void_p(p16.data_ptr()), 0))
    rng = np.random.default_rng(0)
    dout = np.zeros((B, 16), np.float32)
    dout[:, :3] = rng.standard_normal((B, 3)) * 0.05
    dout16 = torch.from_numpy(dout).half().cuda()
    grad = torch.empty(n, dtype=torch.float16, device="cuda")
    L.check(lib.tcnn_module_backward(m, None, ctx, B, None, ctypes.c_void_p(dout16.data_ptr()), ctypes.c_void_p(grad.data_ptr()),
                                     ctypes.c_void_p(pos_d.data_ptr()), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(p16.data_ptr())))
    torch.cuda.synchronize()
    # oracle
    params16 = p16.cpu().numpy().view(np.uint16)
    g = O.grid_cfg(enc, 2)
    nm = O.mlp_n_params(64, 32, 2, 16)
    encv = O.grid_fwd(g, pos, params16[nm:])
    outr, hidden = O.mlp_fwd(64, 32, 2, 16, params16[:nm], encv)
    assert_within_fp16_ulps(O.h2f(out.cpu().numpy().view(np.uint16)), O.h2f(outr))
    d16 = dout16.cpu().numpy().view(np.uint16)
    wg, denc = O.mlp_bwd(64, 32, 2, 16, params16[:nm], encv, hidden, d16)
    gg = O.grid_bwd(g, pos, denc)
    ref = np.concatenate([wg, gg])
    got = grad.float().cpu().numpy()
    assert rel_err(got, ref) <= 1e-3, (rel_err(got, ref), int(np.isnan(got[:nm]).sum()), int(np.isnan(got[nm:]).sum()),
                                       int(np.isnan(ref).sum()), np.nonzero(np.isnan(got))[0][:8])
    # per element: network weights by the term-magnitude bound, grid by its own bound (fp16 outputs)
    assert_wgrad_per_element(got[:nm], wg, O.mlp_wgrad_magnitude(64, 32, 2, 16, params16[:nm], encv, hidden, d16), fp16_out=True)
    _, denc_abs = O.mlp_wgrad_magnitude(64, 32, 2, 16, params16[:nm], encv, hidden, d16, want_dinput=True)
    absum, _ = O.grid_bwd_stats(g, pos, denc_abs)  # abs-backprop magnitude of every update (helpers.trainer_grad_bounds)
    gbound = O.grid_grad_tolerance(g, pos, denc, gg) + 8 * 2.0 ** -10 * absum + 2.0 ** -11 * np.abs(gg) + 2.0 ** -25
    r = np.abs(got[nm:] - gg) / gbound
    k = int(np.argmax(r))
    assert r[k] <= 1.0, (float(r[k]), k, got[nm + k], gg[k], gbound[k])
    lib.tcnn_context_destroy(ctx)
    lib.tcnn_module_destroy(m)


def test_trainer_buffer_views_alias_device_memory(torch_mod):
    """The torch views of trainer buffers (used by the data-parallel all-reduce) alias the
    engine's device memory."""
    torch = torch_mod
    from tinycudann import Trainer
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    pos, tgt = make_batch(1024)
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    g = t.gradients_fp32()
    a = trainer_arrays(t)
    np.testing.assert_array_equal(g.cpu().numpy(), a["g32"])
    g.mul_(2.0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(trainer_arrays(t)["g32"], a["g32"] * 2.0)


def test_overlapped_step_bit_identical_to_sequential(torch_mod):
    """The single-GPU two-launch step (reductions + Adam in the grid backward's epilogue) gives
    bit-identical parameters to training_step(run_optimizer=False) + optimizer_step(); the loss
    sum differs only in summation order."""
    torch = torch_mod
    from tinycudann import Trainer
    ta = Trainer(2, 3, CONFIG_HASH, seed=1337)
    tb = Trainer(2, 3, CONFIG_HASH, seed=1337)
    for s in range(4):
        pos, tgt = make_batch(4096, step=s)
        p, t = torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda()
        ta.training_step(p, t, run_optimizer=True)
        tb.training_step(p, t, run_optimizer=False)
        tb.optimizer_step()
        assert abs(ta.loss() - tb.loss()) <= 1e-6 * abs(tb.loss())
    a, b = trainer_arrays(ta), trainer_arrays(tb)
    np.testing.assert_array_equal(a["w32"], b["w32"])
    np.testing.assert_array_equal(a["w16"], b["w16"])
    np.testing.assert_array_equal(a["g16"], b["g16"])
