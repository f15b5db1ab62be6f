"""ctypes front-end of the CPU restatement (oracle/tcnn_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker / CPU baseline and never as the thing measured or shipped. The product
package (neuralbtf-tiny-cuda-nn_amd/) never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libtcnn_oracle.so")
_lib = None

MAX_LEVELS = 128


class Pcg32(ctypes.Structure):
    _fields_ = [("state", ctypes.c_uint64), ("inc", ctypes.c_uint64)]


class GridCfg(ctypes.Structure):
    _fields_ = [
        ("n_pos_dims", ctypes.c_uint32), ("n_features_per_level", ctypes.c_uint32),
        ("n_levels", ctypes.c_uint32), ("log2_hashmap_size", ctypes.c_uint32),
        ("base_resolution", ctypes.c_uint32), ("per_level_scale", ctypes.c_float),
        ("grid_type", ctypes.c_uint32), ("hash_type", ctypes.c_uint32), ("interpolation", ctypes.c_uint32),
        ("offsets", ctypes.c_uint32 * (MAX_LEVELS + 1)), ("scales", ctypes.c_float * MAX_LEVELS),
        ("res", ctypes.c_uint32 * MAX_LEVELS), ("n_params", ctypes.c_uint32),
        ("opts", ctypes.c_uint32), ("max_level", ctypes.c_float), ("max_level_gpu", ctypes.c_void_p),
        ("stochastic", ctypes.c_uint32),
    ]


class AdamCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in (
        "learning_rate", "beta1", "beta2", "epsilon", "l2_reg", "relative_decay", "absolute_decay",
        "clipping_magnitude", "non_matrix_learning_rate_factor")] + [
        (n, ctypes.c_int) for n in ("adabound", "optimize_matrix_params", "optimize_non_matrix_params")]


class Model(ctypes.Structure):
    _fields_ = [
        ("grid", GridCfg), ("W", ctypes.c_uint32), ("NH", ctypes.c_uint32), ("OUTP", ctypes.c_uint32),
        ("n_output_dims", ctypes.c_uint32), ("activation", ctypes.c_uint32), ("adam", AdamCfg),
        ("n_params", ctypes.c_uint32), ("n_mlp_params", ctypes.c_uint32), ("adam_step", ctypes.c_uint32),
        ("w32", ctypes.POINTER(ctypes.c_float)), ("w16", ctypes.POINTER(ctypes.c_uint16)),
        ("grad16", ctypes.POINTER(ctypes.c_uint16)), ("grad32", ctypes.POINTER(ctypes.c_float)),
        ("m1", ctypes.POINTER(ctypes.c_float)), ("m2", ctypes.POINTER(ctypes.c_float)),
        ("steps", ctypes.POINTER(ctypes.c_uint32)),
        ("enc_type", ctypes.c_uint32), ("n_dims", ctypes.c_uint32), ("n_bins", ctypes.c_uint32), ("IN", ctypes.c_uint32),
        ("enc_scale", ctypes.c_float), ("enc_offset", ctypes.c_float), ("loss_type", ctypes.c_uint32),
    ]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.orc_h2f.restype = ctypes.c_float
        _lib.orc_f2h.restype = ctypes.c_uint16
        _lib.orc_f2h.argtypes = [ctypes.c_float]
        _lib.orc_pcg32_next_float.restype = ctypes.c_float
        _lib.orc_pcg32_next_uint.restype = ctypes.c_uint32
        _lib.orc_pcg32_seed.argtypes = [ctypes.POINTER(Pcg32), ctypes.c_uint64, ctypes.c_uint64]
        _lib.orc_pcg32_advance.argtypes = [ctypes.POINTER(Pcg32), ctypes.c_int64]
        _lib.orc_generate_uniform.argtypes = [ctypes.POINTER(Pcg32), ctypes.c_size_t, ctypes.c_void_p, ctypes.c_float, ctypes.c_float]
        _lib.orc_xavier_uniform.argtypes = [ctypes.POINTER(Pcg32), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_float]
        _lib.orc_random_val.restype = ctypes.c_float
        _lib.orc_random_val.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        _lib.orc_grid_index.restype = ctypes.c_uint32
        _lib.orc_grid_index.argtypes = [ctypes.POINTER(GridCfg), ctypes.c_uint32, ctypes.c_void_p]
        _lib.orc_coherent_prime_hash.restype = ctypes.c_uint32
        _lib.orc_coherent_prime_hash.argtypes = [ctypes.c_uint32, ctypes.c_void_p]
        _lib.orc_grid_fwd.argtypes = [ctypes.POINTER(GridCfg), ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _lib.orc_grid_bwd.argtypes = [ctypes.POINTER(GridCfg), ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _lib.orc_grid_bwd_stats.argtypes = [ctypes.POINTER(GridCfg), ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p]
        _lib.orc_grid_bwd_input.argtypes = [ctypes.POINTER(GridCfg), ctypes.c_uint32] + [ctypes.c_void_p] * 4
        _lib.orc_grid_bwd_bwd.argtypes = [ctypes.POINTER(GridCfg), ctypes.c_uint32] + [ctypes.c_void_p] * 7
        _lib.orc_mlp_n_params.restype = ctypes.c_uint32
        _lib.orc_mlp_fwd.argtypes = [ctypes.c_uint32] * 5 + [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int,
                                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _lib.orc_mlp_bwd.argtypes = [ctypes.c_uint32] * 5 + [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int,
                                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _lib.orc_relative_l2.restype = ctypes.c_double
        _lib.orc_relative_l2.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _lib.orc_l2.restype = ctypes.c_double
        _lib.orc_l2.argtypes = _lib.orc_relative_l2.argtypes
        _lib.orc_adam_step.argtypes = [ctypes.POINTER(AdamCfg), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float, ctypes.c_uint32] + [ctypes.c_void_p] * 6
        _lib.orc_model_init.argtypes = [ctypes.POINTER(Model), ctypes.c_uint32]
        _lib.orc_model_free.argtypes = [ctypes.POINTER(Model)]
        _lib.orc_train_step.restype = ctypes.c_double
        _lib.orc_train_step.argtypes = [ctypes.POINTER(Model), ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        _lib.orc_model_inference.argtypes = [ctypes.POINTER(Model), ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _lib.orc_seed_seq.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        _lib.orc_oneblob_fwd.argtypes = [ctypes.c_uint32] * 3 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        _lib.orc_oneblob_bwd.argtypes = [ctypes.c_uint32] * 3 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        _lib.orc_identity_fwd.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float, ctypes.c_float, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        _lib.orc_hfma.restype = ctypes.c_uint16
        _lib.orc_hfma.argtypes = [ctypes.c_uint16] * 3
        _lib.orc_set_mimic.argtypes = [ctypes.c_int]
        _lib.orc_set_abs_wgrad.argtypes = [ctypes.c_int]
        _lib.orc_act_bwd_output.argtypes = [ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------------------------------------
# config helpers (JSON keys / defaults as in grid.h:1143-1208, src/network.cu:97-138, adam.h)
# ---------------------------------------------------------------------------------------------
GRID_TYPES = {"hash": 0, "dense": 1, "tiled": 2}
HASH_TYPES = {"prime": 0, "coherentprime": 1, "reversedprime": 2}
INTERP = {"nearest": 0, "linear": 1, "smoothstep": 2}


def grid_cfg(enc, n_pos_dims):
    g = GridCfg()
    otype = enc.get("otype", "Grid").lower()
    default_type = "tiled" if otype == "tiledgrid" else ("dense" if otype == "densegrid" else "hash")
    F = int(enc.get("n_features_per_level", 2))
    L = int(enc.get("n_levels", 16))
    base = int(enc.get("base_resolution", 16))
    gtype = enc.get("type", default_type).lower()
    if gtype == "dense":
        default_scale = float(np.exp(np.log(np.float32(256.0) / np.float32(base)) / (L - 1)))
    else:
        default_scale = 2.0
    g.n_pos_dims = n_pos_dims
    g.n_features_per_level = F
    g.n_levels = L
    g.log2_hashmap_size = int(enc.get("log2_hashmap_size", 19))
    g.base_resolution = base
    g.per_level_scale = float(enc.get("per_level_scale", default_scale))
    g.grid_type = GRID_TYPES[gtype]
    g.hash_type = HASH_TYPES[enc.get("hash", "CoherentPrime").lower()]
    g.interpolation = INTERP[enc.get("interpolation", "Linear").lower()]
    g.stochastic = int(bool(enc.get("stochastic_interpolation", False)))
    g.max_level = 1000.0
    g.opts = g.stochastic
    assert lib().orc_grid_init(ctypes.byref(g)) == 0
    return g


def grid_set_max_level(g, max_level, per_point=None):
    """GridEncoding::set_max_level / set_max_level_gpu (grid_interface.h:101-123); per_point must be
    kept alive by the caller while g is used."""
    g.max_level = float(max_level)
    g.max_level_gpu = per_point.ctypes.data if per_point is not None else None
    g.opts = 1


def random_val(seed, idx):
    return lib().orc_random_val(seed, idx)


def adam_cfg(opt):
    c = AdamCfg()
    lib().orc_adam_default(ctypes.byref(c))
    keys = {"learning_rate": "learning_rate", "beta1": "beta1", "beta2": "beta2", "epsilon": "epsilon",
            "l2_reg": "l2_reg", "relative_decay": "relative_decay", "absolute_decay": "absolute_decay",
            "clipping_magnitude": "clipping_magnitude",
            "non_matrix_learning_rate_factor": "non_matrix_learning_rate_factor"}
    for k, f in keys.items():
        if k in opt:
            setattr(c, f, float(opt[k]))
    for k in ("adabound", "optimize_matrix_params", "optimize_non_matrix_params"):
        if k in opt:
            setattr(c, k, int(bool(opt[k])))
    return c


# ---------------------------------------------------------------------------------------------
# numpy-level wrappers
# ---------------------------------------------------------------------------------------------
def f2h(x):
    """fp32 -> fp16 bits (RNE), as uint16 array"""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(x.shape, dtype=np.uint16)
    lib().orc_f2h_array(_p(x), _p(out), ctypes.c_size_t(x.size))
    return out


def h2f(h):
    h = np.ascontiguousarray(h, dtype=np.uint16)
    out = np.empty(h.shape, dtype=np.float32)
    lib().orc_h2f_array(_p(h), _p(out), ctypes.c_size_t(h.size))
    return out


def seed_seq(seeds, n_out):
    s = np.ascontiguousarray(seeds, dtype=np.uint32)
    out = np.empty(n_out, dtype=np.uint32)
    lib().orc_seed_seq(_p(s), len(s), _p(out), n_out)
    return out


def pcg32(initstate, initseq=1):
    r = Pcg32()
    lib().orc_pcg32_seed(ctypes.byref(r), initstate, initseq)
    return r


def generate_uniform(rng, n, lo=0.0, hi=1.0):
    out = np.empty(n, dtype=np.float32)
    lib().orc_generate_uniform(ctypes.byref(rng), n, _p(out), lo, hi)
    return out


def grid_fwd(g, pos, table16):
    """pos: float32 [B, D] (CM), table16 uint16 [n_params] -> enc uint16 [L*F, B] (SoA)"""
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    B = pos.shape[0]
    table16 = np.ascontiguousarray(table16, dtype=np.uint16)
    enc = np.empty((g.n_levels * g.n_features_per_level, B), dtype=np.uint16)
    lib().orc_grid_fwd(ctypes.byref(g), B, _p(pos), _p(table16), _p(enc))
    return enc


def grid_bwd(g, pos, dL_dy16):
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    B = pos.shape[0]
    dL_dy16 = np.ascontiguousarray(dL_dy16, dtype=np.uint16)
    grad = np.zeros(g.n_params, dtype=np.float32)
    lib().orc_grid_bwd(ctypes.byref(g), B, _p(pos), _p(dL_dy16), _p(grad))
    return grad


def grid_bwd_stats(g, pos, dL_dy16):
    """per grid parameter: (sum of |update|, number of updates) of the backward over pos"""
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    B = pos.shape[0]
    dL_dy16 = np.ascontiguousarray(dL_dy16, dtype=np.uint16)
    absum = np.zeros(g.n_params, dtype=np.float32)
    count = np.zeros(g.n_params, dtype=np.uint32)
    lib().orc_grid_bwd_stats(ctypes.byref(g), B, _p(pos), _p(dL_dy16), _p(absum), _p(count))
    return absum, count


def grid_grad_tolerance(g, pos, dL_dy16, ref_grad):
    """Per-element bound |gpu - oracle| of a grid gradient (fp32 [n_params]).

    The GPU sums the exact fp32 products w16 * dL/dy as int32 fixed point with step
    2^-e <= 2^-29.9 * sum_i max_f |dL/dy_i,f| (level sum over at most all B points, grid.hip /
    grid_bin.hip), so each update is off by at most half a step: count * 2^-30.9 * S_level. The
    oracle sums the same products sequentially in fp32: (count - 1) * 2^-24 * sum |update|; the final
    int32 -> fp32 conversion rounds once more (2^-24 relative)."""
    B = pos.shape[0]
    L, F = g.n_levels, g.n_features_per_level
    absum, count = grid_bwd_stats(g, pos, dL_dy16)
    dy = np.abs(h2f(np.asarray(dL_dy16, dtype=np.uint16)).reshape(L, F, B).astype(np.float64))
    S = dy.max(axis=1).sum(axis=1)  # per level
    tol = np.zeros(g.n_params, dtype=np.float64)
    for l in range(L):
        a, b = g.offsets[l] * F, g.offsets[l + 1] * F
        tol[a:b] = count[a:b] * S[l] * 2.0 ** -29.9
    tol += count * 2.0 ** -24 * absum.astype(np.float64) + 2.0 ** -23 * np.abs(np.asarray(ref_grad, dtype=np.float64))
    return tol


def grid_bwd_input(g, pos, table16, dL_dy16):
    """dL/dx float32 [B, D]; dL_dy16 uint16 SoA [L*F, B]"""
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    B = pos.shape[0]
    dx = np.empty(pos.shape, dtype=np.float32)
    lib().orc_grid_bwd_input(ctypes.byref(g), B, _p(pos), _p(np.ascontiguousarray(table16, dtype=np.uint16)),
                             _p(np.ascontiguousarray(dL_dy16, dtype=np.uint16)), _p(dx))
    return dx


def grid_bwd_bwd(g, pos, table16, dL_ddLdx, dL_dy16=None, want_grad=True, want_ddLdy=True, want_dx=True):
    """Second-order grid gradients (grid.h:351-627). dL_ddLdx float32 [B, D]; dL_dy16 uint16 SoA
    [L*F, B] or None. Returns (grad fp32 [n_params] | None, dL_ddLdy fp32 [B, L*F] | None,
    dL_dx fp32 [B, D] | None)."""
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    B = pos.shape[0]
    LF = g.n_levels * g.n_features_per_level
    grad = np.zeros(g.n_params, dtype=np.float32) if want_grad else None
    ddy = np.empty((B, LF), dtype=np.float32) if want_ddLdy else None
    dx = np.empty(pos.shape, dtype=np.float32) if want_dx else None
    dy = None if dL_dy16 is None else np.ascontiguousarray(dL_dy16, dtype=np.uint16)
    lib().orc_grid_bwd_bwd(ctypes.byref(g), B, _p(pos), _p(np.ascontiguousarray(table16, dtype=np.uint16)),
                           _p(np.ascontiguousarray(dL_ddLdx, dtype=np.float32)), _p(dy) if dy is not None else None,
                           _p(grad) if grad is not None else None, _p(ddy) if ddy is not None else None,
                           _p(dx) if dx is not None else None)
    return grad, ddy, dx


def mlp_n_params(W, IN, NH, OUTP):
    return lib().orc_mlp_n_params(W, IN, NH, OUTP)


def mlp_fwd(W, IN, NH, OUTP, params16, x16, input_soa=True, activation=1, want_hidden=True, n_threads=1):
    x16 = np.ascontiguousarray(x16, dtype=np.uint16)
    B = x16.shape[1] if input_soa else x16.shape[0]
    out = np.empty((B, OUTP), dtype=np.uint16)
    hidden = np.empty((NH, B, W), dtype=np.uint16) if want_hidden else None
    lib().orc_mlp_fwd(W, IN, NH, OUTP, activation, _p(np.ascontiguousarray(params16, dtype=np.uint16)), B, _p(x16),
                      int(input_soa), _p(out), _p(hidden) if hidden is not None else None, n_threads)
    return out, hidden


def mlp_bwd(W, IN, NH, OUTP, params16, x16, hidden16, dout16, input_soa=True, activation=1, want_dinput=True, n_threads=1):
    x16 = np.ascontiguousarray(x16, dtype=np.uint16)
    B = x16.shape[1] if input_soa else x16.shape[0]
    wgrad = np.zeros(mlp_n_params(W, IN, NH, OUTP), dtype=np.float32)
    din = np.empty(x16.shape, dtype=np.uint16) if want_dinput else None
    lib().orc_mlp_bwd(W, IN, NH, OUTP, activation, _p(np.ascontiguousarray(params16, dtype=np.uint16)), B, _p(x16),
                      int(input_soa), _p(np.ascontiguousarray(hidden16)), _p(np.ascontiguousarray(dout16, dtype=np.uint16)),
                      _p(wgrad), _p(din) if din is not None else None, n_threads)
    return wgrad, din


def oneblob_fwd(x, n_bins, n_pad=0):
    """x float32 [B, D] -> uint16 AoS [B, D*n_bins + n_pad] (reference kernel_one_blob semantics)"""
    x = np.ascontiguousarray(x, dtype=np.float32)
    B, D = x.shape
    out = np.empty((B, D * n_bins + n_pad), dtype=np.uint16)
    lib().orc_oneblob_fwd(B, D, n_bins, _p(x), _p(out), D * n_bins + n_pad, n_pad)
    return out


def oneblob_bwd(x, n_bins, dy16):
    """dL/dx float32 [B, D] from dL/dy uint16 AoS [B, stride]"""
    x = np.ascontiguousarray(x, dtype=np.float32)
    dy16 = np.ascontiguousarray(dy16, dtype=np.uint16)
    B, D = x.shape
    dx = np.empty((B, D), dtype=np.float32)
    lib().orc_oneblob_bwd(B, D, n_bins, _p(x), _p(dy16), dy16.shape[1], _p(dx))
    return dx


def identity_fwd(x, scale=1.0, offset=0.0, n_pad=0):
    x = np.ascontiguousarray(x, dtype=np.float32)
    B, D = x.shape
    out = np.empty((B, D + n_pad), dtype=np.uint16)
    lib().orc_identity_fwd(B, D, scale, offset, _p(x), _p(out), D + n_pad, n_pad)
    return out


def relative_l2(pred16, target, loss_scale=128.0, want_values=False):
    """pred16 uint16 [B, stride] CM; target float32 [B, dims]"""
    pred16 = np.ascontiguousarray(pred16, dtype=np.uint16)
    target = np.ascontiguousarray(target, dtype=np.float32)
    B, stride = pred16.shape
    dims = target.shape[1]
    grads = np.empty_like(pred16)
    values = np.empty((B, stride), dtype=np.float32) if want_values else None
    s = lib().orc_relative_l2(B, stride, dims, loss_scale, _p(pred16), _p(target),
                              _p(values) if values is not None else None, _p(grads))
    return s, grads, values


def adam_step(cfg, n_matrix, loss_scale, current_step, w32, w16, grad16, m1, m2, steps):
    lib().orc_adam_step(ctypes.byref(cfg), len(w32), n_matrix, loss_scale, current_step,
                        _p(w32), _p(w16), _p(grad16), _p(m1), _p(m2), _p(steps))


ACTIVATIONS = ["none", "relu", "leakyrelu", "exponential", "sine", "sigmoid", "squareplus", "softplus", "tanh"]


def act_code(name):
    """Activation enum value (common.h:126-136) of a config string (case-insensitive)"""
    return ACTIVATIONS.index(name.lower())


def set_mimic(on):
    """reference-mimic fp16 accumulation on / off, process-wide"""
    lib().orc_set_mimic(1 if on else 0)


def mlp_wgrad_magnitude(W, IN, NH, OUTP, params16, x16, hidden16, dout16, input_soa=True, activation=1, n_threads=1,
                        want_dinput=False):
    """sum_i |delta_i| |a_i| per MLP weight, the deltas propagated through |W| with the forward's
    activation masks (abs-backprop): the per-element scale of the weight gradient's tolerance
    (tests/helpers.assert_wgrad_per_element). want_dinput: also the abs-backprop dL/dinput (fp16), the
    scale of a dL/dinput element's tolerance. Returns wg, or (wg, dinput) with want_dinput."""
    lib().orc_set_abs_wgrad(1)
    try:
        wg, din = mlp_bwd(W, IN, NH, OUTP, params16, x16, hidden16, dout16, input_soa=input_soa, activation=activation,
                          want_dinput=want_dinput, n_threads=n_threads)
    finally:
        lib().orc_set_abs_wgrad(0)
    return (wg, din) if want_dinput else wg


def act_bwd_output(act, out16, g16):
    """in-place output-activation transfer (act: hidden | output << 8) of fp16 dL/dout given fp16 outputs"""
    g16 = np.ascontiguousarray(g16, dtype=np.uint16)
    out16 = np.ascontiguousarray(out16, dtype=np.uint16)
    lib().orc_act_bwd_output(act, ctypes.c_size_t(g16.size), _p(out16), _p(g16))
    return g16


class OracleModel:
    """Trainer<float,__half,__half> over NetworkWithInputEncoding<Grid | OneBlob | Identity,
    FullyFusedMLP> on the CPU (encoding padded to 16 columns, network.cu:76-95)."""

    def __init__(self, config, n_input_dims, n_output_dims, seed=1337):
        self.m = Model()
        enc, net, opt = config["encoding"], config["network"], config.get("optimizer", {})
        eo = enc.get("otype", "OneBlob").lower()
        self.m.n_dims = n_input_dims
        if eo == "oneblob":
            self.m.enc_type = 1
            self.m.n_bins = int(enc.get("n_bins", 16))
            self.m.IN = (n_input_dims * self.m.n_bins + 15) // 16 * 16
        elif eo == "identity":
            self.m.enc_type = 2
            self.m.enc_scale = float(enc.get("scale", 1.0))
            self.m.enc_offset = float(enc.get("offset", 0.0))
            self.m.IN = (n_input_dims + 15) // 16 * 16
        else:
            self.m.enc_type = 0
            self.m.grid = grid_cfg(enc, n_input_dims)
        self.m.W = int(net.get("n_neurons", 128))
        self.m.NH = int(net.get("n_hidden_layers", 5))
        self.m.n_output_dims = n_output_dims
        self.m.OUTP = (n_output_dims + 15) // 16 * 16
        self.m.activation = act_code(net.get("activation", "ReLU")) | (act_code(net.get("output_activation", "None")) << 8)
        self.m.adam = adam_cfg(opt)
        lo = config.get("loss", {}).get("otype", "RelativeL2").lower()
        self.m.loss_type = {"relativel2": 0, "l2": 1}[lo]
        assert lib().orc_model_init(ctypes.byref(self.m), seed) == 0
        self.n_params = self.m.n_params
        self.n_mlp_params = self.m.n_mlp_params

    def __del__(self):
        try:
            lib().orc_model_free(ctypes.byref(self.m))
        except Exception:
            pass

    def _arr(self, ptr, dtype):
        return np.ctypeslib.as_array(ptr, shape=(self.n_params,)).view(dtype)

    @property
    def w32(self):
        return np.ctypeslib.as_array(self.m.w32, shape=(self.n_params,))

    @property
    def w16(self):
        return np.ctypeslib.as_array(self.m.w16, shape=(self.n_params,))

    @property
    def grad16(self):
        return np.ctypeslib.as_array(self.m.grad16, shape=(self.n_params,))

    @property
    def grad32(self):
        return np.ctypeslib.as_array(self.m.grad32, shape=(self.n_params,))

    def train_step(self, pos, target, run_optimizer=True, n_threads=1):
        pos = np.ascontiguousarray(pos, dtype=np.float32)
        target = np.ascontiguousarray(target, dtype=np.float32)
        return lib().orc_train_step(ctypes.byref(self.m), pos.shape[0], _p(pos), _p(target), int(run_optimizer), n_threads)

    def inference(self, pos, n_threads=1):
        pos = np.ascontiguousarray(pos, dtype=np.float32)
        out = np.empty((pos.shape[0], self.m.OUTP), dtype=np.uint16)
        lib().orc_model_inference(ctypes.byref(self.m), pos.shape[0], _p(pos), _p(out), n_threads)
        return out


def l2(pred16, target, loss_scale=128.0, want_values=False):
    """L2 loss (losses/l2.h:40-76); same layouts as relative_l2"""
    pred16 = np.ascontiguousarray(pred16, dtype=np.uint16)
    target = np.ascontiguousarray(target, dtype=np.float32)
    B, stride = pred16.shape
    dims = target.shape[1]
    grads = np.empty_like(pred16)
    values = np.empty((B, stride), dtype=np.float32) if want_values else None
    s = lib().orc_l2(B, stride, dims, loss_scale, _p(pred16), _p(target),
                     _p(values) if values is not None else None, _p(grads))
    return s, grads, values
