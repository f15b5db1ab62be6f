"""GPU parity of the grid backward, per element, including the large-table (binned) path.

BASELINE configs[2] as written: HashGrid L16 F2 log2_T=19 per_level_scale=2.0 (the DOCUMENTATION.md
defaults SURVEY §8(d) C3 names) + FullyFusedMLP 64x2. Its levels 4..15 (65,536 .. 524,288 entries)
do not fit a CU's LDS and run through the binned backward (csrc/grid_bin.hip); levels 0..3 run
through the LDS items (csrc/grid.hip). Reference: kernel_grid_backward, grid.h:214-320.

Tolerance (stated, per element, no relative-L2 aggregate): the GPU sums the exact fp32 products
(half)w * dL/dy as int32 fixed point whose step is <= 2^-29.9 * sum_i max_f |dL/dy_i| of the level;
the oracle sums the same products in fp32. oracle.grid_grad_tolerance() gives the bound
count * step + count * 2^-24 * sum|update| + 2^-23 |ref| per parameter; fp16 outputs of the Module
API add half an fp16 ulp. The reference itself accumulates in fp16 atomics (grid.h:252-255), whose
error is ~2^-11 of the running sum per add -- far above this bound.
"""
import copy
import ctypes
import json
import os

import numpy as np
import pytest

from helpers import CONFIG_HASH, make_batch, trainer_arrays
from oracle import oracle as O

pytestmark = pytest.mark.gpu

ENC_T19 = dict(CONFIG_HASH["encoding"], log2_hashmap_size=19, per_level_scale=2.0)
CONFIG_T19 = dict(copy.deepcopy(CONFIG_HASH), encoding=ENC_T19)


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available()
    return torch


def _vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _module_grad(torch, enc, D, pos, dy_aos16, table16=None):
    """GridEncoding Module forward + backward (tcnn_module_*): fp16 grads [n_params]"""
    from tinycudann import _lib as L
    lib = L.lib()
    m = L.check_ptr(lib.tcnn_create_encoding(D, json.dumps(enc).encode(), 1))
    try:
        B = pos.shape[0]
        W = lib.tcnn_module_n_output_dims(m)
        n = lib.tcnn_module_n_params(m)
        if table16 is None:
            p32 = torch.zeros(n, dtype=torch.float32, device="cuda")
            L.check(lib.tcnn_module_initialize_params(m, 1337, _vp(p32), 1.0))
            p16 = p32.half()
        else:
            p16 = torch.from_numpy(table16.view(np.float16)).cuda()
        pos_d = torch.from_numpy(np.ascontiguousarray(pos)).cuda()
        out = torch.empty(B, W, dtype=torch.float16, device="cuda")
        ctx = L.check_ptr(lib.tcnn_module_forward(m, None, B, _vp(pos_d), _vp(out), _vp(p16), 0))
        dy_full = np.zeros((B, W), dtype=np.uint16)
        dy_full[:, :dy_aos16.shape[1]] = dy_aos16
        dy_d = torch.from_numpy(dy_full.view(np.float16)).cuda()
        grad = torch.empty(n, dtype=torch.float16, device="cuda")
        L.check(lib.tcnn_module_backward(m, None, ctx, B, None, _vp(dy_d), _vp(grad), _vp(pos_d), _vp(out), _vp(p16)))
        torch.cuda.synchronize()
        lib.tcnn_context_destroy(ctx)
        return grad.float().cpu().numpy()
    finally:
        lib.tcnn_module_destroy(m)


def _check_grid_grad(got, ref, tol, fp16_out, what):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    if fp16_out:
        tol = tol + 2.0 ** -11 * (np.abs(ref) + tol) + 2.0 ** -25
    err = np.abs(got - ref)
    bad = np.flatnonzero(err > tol)
    worst = int(np.argmax(err / np.maximum(tol, 1e-30)))
    msg = (f"{what}: {bad.size} of {ref.size} elements outside the bound; worst p={worst} got={got[worst]!r} "
           f"ref={ref[worst]!r} tol={tol[worst]!r}; max|err|={err.max():.3e}")
    assert bad.size == 0, msg
    return float(err.max())


def _random_dy(B, L, F, seed, scale=1.0):
    rng = np.random.default_rng(seed)
    dy = (rng.standard_normal((B, L * F)) * scale).astype(np.float16)
    return dy.view(np.uint16)


def _module_case(torch, enc, D, B, seed=5, pos=None, dy=None):
    g = O.grid_cfg(enc, D)
    L, F = g.n_levels, g.n_features_per_level
    if pos is None:
        r = O.pcg32(seed)
        pos = O.generate_uniform(r, D * B).reshape(B, D)
    if dy is None:
        dy = _random_dy(B, L, F, seed)
    got = _module_grad(torch, enc, D, pos, dy)
    dy_soa = np.ascontiguousarray(dy.T)
    ref = O.grid_bwd(g, pos, dy_soa)
    tol = O.grid_grad_tolerance(g, pos, dy_soa, ref)
    return got, ref, tol, g


@pytest.mark.parametrize("B", [256, 4096])
def test_module_grad_log2t19_per_element(torch_mod, B):
    got, ref, tol, _ = _module_case(torch_mod, ENC_T19, 2, B)
    _check_grid_grad(got, ref, tol, True, f"log2T=19 B={B}")


def test_module_grad_config_hash_binned_all(torch_mod, monkeypatch):
    """config_hash as-is with every level that does not fit whole sent through the binned path"""
    monkeypatch.setenv("TCNN_GRID_BIN", "all")
    got, ref, tol, _ = _module_case(torch_mod, CONFIG_HASH["encoding"], 2, 4096)
    _check_grid_grad(got, ref, tol, True, "config_hash TCNN_GRID_BIN=all")


def test_module_grad_config_hash_lds_per_element(torch_mod):
    got, ref, tol, _ = _module_case(torch_mod, CONFIG_HASH["encoding"], 2, 4096)
    _check_grid_grad(got, ref, tol, True, "config_hash LDS items")


@pytest.mark.parametrize("enc_name", ["config_hash", "log2t19"])
def test_outlier_dy_keeps_resolution(torch_mod, enc_name):
    """One dL/dy 1000x the others in a chunk: the fixed-point step follows sum |dL/dy|, so the
    other entries keep their resolution (a max-based scale would lose ~2^10 of it)."""
    enc = CONFIG_HASH["encoding"] if enc_name == "config_hash" else ENC_T19
    B = 4096
    g = O.grid_cfg(enc, 2)
    dy = _random_dy(B, g.n_levels, g.n_features_per_level, 11).view(np.float16).copy()
    dy[123, :] = np.float16(1000.0)
    got, ref, tol, _ = _module_case(torch_mod, enc, 2, B, seed=11, dy=dy.view(np.uint16))
    _check_grid_grad(got, ref, tol, True, f"{enc_name} with an outlier dL/dy")
    # the bound itself stays fine-grained: median tolerance relative to |ref| well below fp16 resolution
    nz = np.abs(ref) > 0
    assert np.median(tol[nz] / np.abs(ref[nz])) < 2.0 ** -14


@pytest.mark.parametrize("enc_name", ["config_hash", "log2t19"])
def test_positions_outside_unit_square(torch_mod, enc_name):
    """x in [-0.5, 1.5]: dense levels wrap with index % size (common_device.h:706) in the backward too"""
    enc = CONFIG_HASH["encoding"] if enc_name == "config_hash" else ENC_T19
    B = 4096
    r = O.pcg32(21)
    pos = (O.generate_uniform(r, 2 * B).reshape(B, 2) * 2.0 - 0.5).astype(np.float32)
    got, ref, tol, _ = _module_case(torch_mod, enc, 2, B, seed=21, pos=pos)
    _check_grid_grad(got, ref, tol, True, f"{enc_name} x in [-0.5, 1.5]")


@pytest.mark.parametrize("enc_name", ["config_hash", "log2t19"])
def test_nonfinite_dy_propagates(torch_mod, enc_name):
    """A NaN dL/dy makes its level's gradient NaN (the reference's fp16 atomics carry it); other
    levels stay finite."""
    enc = CONFIG_HASH["encoding"] if enc_name == "config_hash" else ENC_T19
    B = 4096
    g = O.grid_cfg(enc, 2)
    L, F = g.n_levels, g.n_features_per_level
    dy = _random_dy(B, L, F, 3).view(np.float16).copy()
    lev = L - 1
    dy[77, lev * F:(lev + 1) * F] = np.float16("nan")
    got, _, _, g = _module_case(torch_mod, enc, 2, B, seed=3, dy=dy.view(np.uint16))
    a, b = g.offsets[lev] * F, g.offsets[lev + 1] * F
    assert np.isnan(got[a:b]).any()
    assert np.isfinite(got[:a]).all()


GRID_VARIANTS = [
    # (D, enc overrides) -- §8(f) rank 4: dims, features per level, grid types, hashes, interpolation
    (3, dict(n_levels=8, n_features_per_level=2, log2_hashmap_size=15, base_resolution=8, per_level_scale=1.5)),
    (4, dict(n_levels=6, n_features_per_level=2, log2_hashmap_size=14, base_resolution=4, per_level_scale=1.5)),
    (2, dict(n_levels=8, n_features_per_level=1, log2_hashmap_size=17, base_resolution=16, per_level_scale=2.0)),
    (2, dict(n_levels=8, n_features_per_level=4, log2_hashmap_size=16, base_resolution=16, per_level_scale=2.0)),
    (2, dict(n_levels=6, n_features_per_level=8, log2_hashmap_size=15, base_resolution=16, per_level_scale=2.0)),
    (3, dict(n_levels=6, n_features_per_level=4, log2_hashmap_size=18, base_resolution=16, per_level_scale=2.0)),
    (2, dict(type="Dense", n_levels=8, n_features_per_level=2, base_resolution=16, per_level_scale=1.6)),
    (3, dict(type="Tiled", n_levels=6, n_features_per_level=2, base_resolution=24, per_level_scale=1.5)),
    (2, dict(n_levels=8, n_features_per_level=2, log2_hashmap_size=17, hash="Prime", per_level_scale=2.0)),
    (2, dict(n_levels=8, n_features_per_level=2, log2_hashmap_size=17, hash="ReversedPrime", per_level_scale=2.0)),
    (2, dict(n_levels=8, n_features_per_level=2, log2_hashmap_size=17, interpolation="Smoothstep", per_level_scale=2.0)),
    (2, dict(n_levels=8, n_features_per_level=2, log2_hashmap_size=17, interpolation="Nearest", per_level_scale=2.0)),
]


@pytest.mark.parametrize("D,over", GRID_VARIANTS, ids=[f"D{d}-" + "-".join(f"{k}{v}" for k, v in o.items()) for d, o in GRID_VARIANTS])
def test_grid_variant_forward_and_grad(torch_mod, D, over):
    """forward bit-exact and per-element gradient vs the oracle for each grid option (grid.h:1143-1208)"""
    torch = torch_mod
    from tinycudann import _lib as L
    lib = L.lib()
    enc = dict({"otype": "HashGrid", "type": "Hash", "interpolation": "Linear"}, **over)
    B = 2048
    g = O.grid_cfg(enc, D)
    r = O.pcg32(9)
    pos = O.generate_uniform(r, D * B).reshape(B, D)
    m = L.check_ptr(lib.tcnn_create_encoding(D, json.dumps(enc).encode(), 1))
    n = lib.tcnn_module_n_params(m)
    assert n == g.n_params
    p32 = torch.zeros(n, dtype=torch.float32, device="cuda")
    L.check(lib.tcnn_module_initialize_params(m, 1337, _vp(p32), 1.0))
    p16 = (p32 * 5000.0).half().contiguous()
    W = lib.tcnn_module_n_output_dims(m)
    out = torch.empty(B, W, dtype=torch.float16, device="cuda")
    pos_d = torch.from_numpy(pos).cuda()
    L.check(lib.tcnn_module_inference(m, None, B, _vp(pos_d), _vp(out), _vp(p16)))
    torch.cuda.synchronize()
    lib.tcnn_module_destroy(m)
    table = p16.cpu().numpy().view(np.uint16)
    ref_out = O.grid_fwd(g, pos, table)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16)[:, :ref_out.shape[0]].T, ref_out)
    dy = _random_dy(B, g.n_levels, g.n_features_per_level, 4)
    got = _module_grad(torch, enc, D, pos, dy, table16=table)
    dy_soa = np.ascontiguousarray(dy.T)
    ref = O.grid_bwd(g, pos, dy_soa)
    tol = O.grid_grad_tolerance(g, pos, dy_soa, ref)
    _check_grid_grad(got, ref, tol, True, f"D={D} {over}")


def _t19_trainer(torch):
    from tinycudann import Trainer
    t = Trainer(2, 3, CONFIG_T19, seed=1337)
    assert t.engine == "fused"
    return t


@pytest.mark.parametrize("B", [256, 4096])
def test_trainer_log2t19_gradients(torch_mod, B):
    """configs[2] as written: fused engine + binned grid backward; run_optimizer=False gradients"""
    torch = torch_mod
    t = _t19_trainer(torch)
    om = O.OracleModel(CONFIG_T19, 2, 3, seed=1337)
    np.testing.assert_array_equal(trainer_arrays(t)["w32"], om.w32)
    pos, tgt = make_batch(B)
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    loss_gpu = t.loss()
    loss_ref = om.train_step(pos, tgt, run_optimizer=False)
    assert abs(loss_gpu - loss_ref) <= 1e-3 * abs(loss_ref), (loss_gpu, loss_ref)
    a = trainer_arrays(t)
    nm = om.n_mlp_params
    # network gradients: fp32 MFMA vs fp32 CPU order -> relative L2 (as test_gpu_parity)
    from helpers import rel_err
    assert rel_err(a["g32"][:nm], om.grad32[:nm]) <= 1e-3
    assert rel_err(a["g32"][nm:], om.grad32[nm:]) <= 1e-3
    # per element: dL/d(encoding) comes from each side's MLP backward, so the grid bound adds 8 fp16
    # ulps of every update to the grid backward's own bound (helpers.trainer_grad_bounds)
    # (on a batch clear of the ReLU boundaries, helpers.relu_margin_ok)
    from helpers import assert_trainer_grads_per_element, relu_safe_grid_batch, trainer_grad_bounds
    t2 = _t19_trainer(torch)
    om2 = O.OracleModel(CONFIG_T19, 2, 3, seed=1337)
    pos, tgt = relu_safe_grid_batch(CONFIG_T19, om2.w16, B)
    t2.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    om2.train_step(pos, tgt, run_optimizer=False)
    a2 = trainer_arrays(t2)
    mag, gb = trainer_grad_bounds(CONFIG_T19, a2["w16"], pos, tgt)
    assert_trainer_grads_per_element(a2["g32"], om2.grad32, nm, mag, gb)


def test_trainer_log2t19_adam_step(torch_mod):
    """Adam applied inside the binned accumulate pass == the oracle's Adam on the same fp16 grads"""
    torch = torch_mod
    t = _t19_trainer(torch)
    om = O.OracleModel(CONFIG_T19, 2, 3, seed=1337)
    pos, tgt = make_batch(4096)
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=True)
    a = trainer_arrays(t)
    w32, w16 = om.w32.copy(), om.w16.copy()
    m1 = np.zeros(om.n_params, np.float32)
    m2 = np.zeros_like(m1)
    steps = np.zeros(om.n_params, np.uint32)
    O.adam_step(om.m.adam, om.n_mlp_params, 128.0, 1, w32, w16, a["g16"], m1, m2, steps)
    np.testing.assert_array_equal(a["w32"], w32)  # bit for bit (the binned levels' Adam runs in k_grid_acc)
    np.testing.assert_array_equal(a["w16"], w16)


def test_trainer_log2t19_sequential_equals_overlapped(torch_mod):
    """training_step(run_optimizer=False) + optimizer_step() == the overlapped step, bit for bit"""
    torch = torch_mod
    t1 = _t19_trainer(torch)
    t2 = _t19_trainer(torch)
    for s in range(3):
        pos, tgt = make_batch(4096, step=s)
        p, q = torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda()
        t1.training_step(p, q, run_optimizer=True)
        t2.training_step(p, q, run_optimizer=False)
        t2.optimizer_step()
    a1, a2 = trainer_arrays(t1), trainer_arrays(t2)
    np.testing.assert_array_equal(a1["w32"], a2["w32"])


def test_full_size_log2t19_properties(torch_mod):
    """B = 2^18 (the bench size) through the Module API: bit-identical on a rerun (integer sums are
    order-independent), and per level the gradient mass equals sum_i dL/dy_i * sum_c (half)w_c
    within the fixed-point bound."""
    torch = torch_mod
    B = 1 << 18
    g = O.grid_cfg(ENC_T19, 2)
    L, F = g.n_levels, g.n_features_per_level
    r = O.pcg32(99)
    pos = O.generate_uniform(r, 2 * B).reshape(B, 2)
    dy = _random_dy(B, L, F, 99)
    g1 = _module_grad(torch, ENC_T19, 2, pos, dy)
    g2 = _module_grad(torch, ENC_T19, 2, pos, dy)
    np.testing.assert_array_equal(g1.view(np.uint32), g2.view(np.uint32))
    # mass per level and feature: sum over entries of the gradient = sum over points of dy * W_i,
    # W_i = sum of the four fp16 corner weights (float64 here; fp16 rounding of the stored grads ->
    # compare with 2^-10 relative slack on the absolute mass)
    dyf = O.h2f(dy).astype(np.float64).reshape(B, L, F)
    for l in range(L):
        s = np.float32(g.scales[l])
        p = (pos.astype(np.float64) * float(s) + 0.5).astype(np.float32)  # ~ fmaf(scale, x, 0.5)
        fr = (p - np.floor(p)).astype(np.float32)
        w = np.zeros(B)
        for c in range(4):
            wx = fr[:, 0] if c & 1 else (np.float32(1) - fr[:, 0])
            wy = fr[:, 1] if c & 2 else (np.float32(1) - fr[:, 1])
            w += (wx * wy).astype(np.float32).astype(np.float16).astype(np.float64)
        a, b = g.offsets[l] * F, g.offsets[l + 1] * F
        got = g1[a:b].astype(np.float64).reshape(-1, F).sum(axis=0)
        exp = (dyf[:, l, :] * w[:, None]).sum(axis=0)
        absmass = (np.abs(dyf[:, l, :]) * w[:, None]).sum(axis=0)
        assert np.all(np.abs(got - exp) <= 2.0 ** -9 * absmass + 1e-3), (l, got, exp)
