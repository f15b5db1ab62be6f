"""Shared test helpers: seeded synthetic batches (reference sample's pcg32{1337} strided RNG for
positions, an analytic RGB field for targets) and device<->host plumbing for trainer buffers."""
import ctypes
import json
import os

import numpy as np

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CONFIG_HASH = json.load(open(os.path.join(GOLD, "config_hash.json")))
CONFIG_ONEBLOB = json.load(open(os.path.join(GOLD, "config_oneblob.json")))


def rgb_field(pos):
    """Smooth synthetic RGB image on [0,1)^2 (stands in for albert.jpg's bilinear texture fetch)."""
    x, y = pos[:, 0].astype(np.float64), pos[:, 1].astype(np.float64)
    r = 0.5 + 0.5 * np.sin(9.0 * x) * np.cos(7.0 * y)
    g = 0.5 + 0.4 * np.sin(23.0 * x * y + 1.0)
    b = 0.5 + 0.3 * np.cos(31.0 * x) * np.sin(17.0 * y) + 0.1 * ((x * 40).astype(np.int64) % 2)
    return np.stack([r, g, b], axis=1).astype(np.float32)


def make_batch(B, seed=1337, step=0):
    """positions [B,2] from pcg32{seed} in generate_random_uniform order (random.h:39-70),
    advanced by `step` batches; targets from rgb_field."""
    r = O.pcg32(seed)
    if step:
        O.lib().orc_pcg32_advance(ctypes.byref(r), 2 * B * step)
    pos = O.generate_uniform(r, 2 * B).reshape(B, 2)
    return pos, rgb_field(pos)


_hip = None


def hip():
    global _hip
    if _hip is None:
        import torch  # noqa: F401  (loads the HIP runtime torch uses; same SONAME as ours)
        _hip = ctypes.CDLL("libamdhip64.so.7")
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipDeviceSynchronize.argtypes = []
    return _hip


def d2h(ptr, n, dtype):
    """copy n elements of dtype from a device pointer to a numpy array"""
    out = np.empty(n, dtype=dtype)
    hip().hipDeviceSynchronize()
    rc = hip().hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr), out.nbytes, 2)  # D2H
    assert rc == 0
    return out


def trainer_arrays(t):
    from tinycudann import _lib as L
    lib = L.lib()
    n = t.n_params
    return {
        "w32": d2h(lib.tcnn_trainer_params_fp32(t.h), n, np.float32),
        "w16": d2h(lib.tcnn_trainer_params(t.h), n, np.uint16),
        "g16": d2h(lib.tcnn_trainer_param_gradients(t.h), n, np.uint16),
        "g32": d2h(lib.tcnn_trainer_gradients_fp32(t.h), n, np.float32),
    }


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def assert_within_fp16_ulps(got, ref, n_ulp=4):
    """max |got - ref| <= n_ulp fp16 ulps at the output scale (max |ref|): the network-output bar
    (fp32 MFMA accumulation vs the oracle's CPU summation order). A fixed absolute tolerance above
    the output scale would accept unwritten (zero) rows -- the seed-1337 init gives outputs ~1e-5."""
    scale = float(np.abs(ref).max())
    assert scale > 0
    ulp = float(np.spacing(np.float16(scale)))
    err = float(np.abs(np.asarray(got, np.float64) - np.asarray(ref, np.float64)).max())
    assert err <= n_ulp * ulp, (err, ulp, scale)


def assert_wgrad_per_element(got, ref, mag, ulps=8, fp16_out=False, floor_rel=1e-6):
    """Per-element bound of an MLP weight gradient dW = sum_i delta_i a_i. Between the HIP kernels
    (fp32 MFMA) and the oracle (fp32 CPU order) a term's fp16 activation or delta can round to the
    neighbouring fp16 value, so each term may differ by a few fp16 ulps (2^-10 relative):
    |got - ref| <= ulps * 2^-10 * mag + floor_rel * max|ref| (+ 2^-11 |ref| when got was rounded to
    fp16), mag = sum_i |delta_i a_i| (oracle.mlp_wgrad_magnitude). The fp32 summation error of either
    side (K * 2^-24 relative) is far below this."""
    got, ref, mag = (np.asarray(v, np.float64) for v in (got, ref, mag))
    bound = ulps * 2.0 ** -10 * mag + floor_rel * np.abs(ref).max()
    if fp16_out:
        bound += 2.0 ** -11 * np.abs(ref) + 2.0 ** -25  # fp16 rounding (subnormals: half the smallest step)
    r = np.abs(got - ref) / bound
    k = int(np.argmax(r))
    assert r[k] <= 1.0, (float(r[k]), k, got[k], ref[k], mag[k])
    return float(r[k])


def relu_margin_ok(W, IN, NH, params16, x_rows, tau=2.0 ** -11, check_output=False):
    """Per sample: True when no hidden pre-activation of the ReLU MLP lies within tau * sum_k |w_k a_k|
    of zero. At such a boundary fp32-MFMA and CPU summation orders may legitimately take different
    ReLU branches (a discrete difference no rounding bound covers); per-element gradient checks run on
    batches of samples clear of it, the aggregate checks on every sample. tau = 2^-11 covers one fp16
    ulp of difference in any single input term (|w_k| ulp(a_k) <= 2^-11 |w_k a_k|) plus the fp32
    summation-order noise. check_output (loss-driven steps): also False when the output's fp16 rounding
    is within 2^-18 sum |w a| of a rounding boundary. x_rows: float [B][IN] (the fp16 encoded input values)."""
    p = O.h2f(np.asarray(params16, np.uint16)).astype(np.float64)
    mats, off, k = [], 0, IN
    for _ in range(NH):
        mats.append(p[off:off + W * k].reshape(W, k))
        off += W * k
        k = W
    a = np.asarray(x_rows, np.float64)
    ok = np.ones(a.shape[0], bool)
    for Wm in mats:
        z = a @ Wm.T
        mag = np.abs(a) @ np.abs(Wm).T
        ok &= np.all(np.abs(z) >= tau * mag, axis=1)
        a = np.maximum(z, 0.0).astype(np.float16).astype(np.float64)  # the fp16 post-activation
    if not check_output:
        return ok
    # the output's fp16 rounding: both sides must round to the same value, else the loss gradient
    # 2 (p - t) / (p^2 + 0.01) of a sample with a small error p - t changes by a large factor
    Wo = p[off:off + 16 * k].reshape(16, k)
    y, ymag = a @ Wo.T, np.abs(a) @ np.abs(Wo).T
    eps = 2.0 ** -18 * ymag
    ok &= np.all((y - eps).astype(np.float16) == (y + eps).astype(np.float16), axis=1)
    return ok


def relu_safe_grid_batch(cfg, params16, B, seed=1337, step=0):
    """A B-point batch (make_batch order) of samples clear of the ReLU boundaries (relu_margin_ok) for
    the grid-encoded network of cfg at params16."""
    W, NH = cfg["network"]["n_neurons"], cfg["network"]["n_hidden_layers"]
    g = O.grid_cfg(cfg["encoding"], 2)
    IN = g.n_levels * g.n_features_per_level
    nm = O.mlp_n_params(W, IN, NH, 16)
    p16 = np.asarray(params16, np.uint16)
    pos, tgt = make_batch(4 * B, seed=seed, step=step)
    enc = O.h2f(O.grid_fwd(g, pos, p16[nm:])).T  # [B][IN]
    ok = relu_margin_ok(W, IN, NH, p16[:nm], enc, check_output=True)
    assert ok.sum() >= B, ok.sum()
    idx = np.nonzero(ok)[0][:B]
    return np.ascontiguousarray(pos[idx]), np.ascontiguousarray(tgt[idx])


def trainer_grad_bounds(cfg, params16, pos, tgt, n_threads=4):
    """The oracle's intermediates of one training step on (pos, tgt) with parameters params16 (grid
    encoding + FullyFusedMLP, RelativeL2): returns (mlp magnitude, grid bound) for per-element checks of
    the trainer's fp32 gradient sums. Grid bound = the grid backward's own bound for the oracle's
    dL/d(encoding) (oracle.grid_grad_tolerance) + 8 fp16 ulps of every update's abs-backprop magnitude
    (the GPU's dL/d(encoding) comes from its own MLP backward: an fp16 delta upstream that rounds to
    its neighbouring value moves it by up to an ulp of that magnitude, cancellation included)."""
    enc_cfg, net = cfg["encoding"], cfg["network"]
    W, NH = net["n_neurons"], net["n_hidden_layers"]
    g = O.grid_cfg(enc_cfg, pos.shape[1])
    IN = g.n_levels * g.n_features_per_level
    nm = O.mlp_n_params(W, IN, NH, 16)
    p16 = np.asarray(params16, np.uint16)
    enc = O.grid_fwd(g, pos, p16[nm:])
    out16, hidden = O.mlp_fwd(W, IN, NH, 16, p16[:nm], enc, n_threads=n_threads)
    _, dout, _ = O.relative_l2(out16, tgt)
    mag, denc_abs = O.mlp_wgrad_magnitude(W, IN, NH, 16, p16[:nm], enc, hidden, dout, n_threads=n_threads, want_dinput=True)
    _, denc = O.mlp_bwd(W, IN, NH, 16, p16[:nm], enc, hidden, dout, n_threads=n_threads)
    ref_grid = O.grid_bwd(g, pos, denc)
    absum, _ = O.grid_bwd_stats(g, pos, denc_abs)
    grid_bound = O.grid_grad_tolerance(g, pos, denc, ref_grid) + 8 * 2.0 ** -10 * absum.astype(np.float64)
    return mag, grid_bound


def assert_trainer_grads_per_element(g32, ref32, n_mlp, mag, grid_bound):
    assert_wgrad_per_element(g32[:n_mlp], ref32[:n_mlp], mag)
    got, ref = np.asarray(g32[n_mlp:], np.float64), np.asarray(ref32[n_mlp:], np.float64)
    r = np.abs(got - ref) / (grid_bound + 1e-30)
    k = int(np.argmax(r))
    assert r[k] <= 1.0, (float(r[k]), k, got[k], ref[k], grid_bound[k])
