"""Oracle pinning: the CPU restatement (oracle/) against the reference's own compiled sources
(tests/golden/ref_known_answers.json, produced by oracle/_ref from /root/reference's pcg32.h +
std::seed_seq) and the SURVEY.md §8(c) known answers."""
import ctypes
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KA = json.load(open(os.path.join(GOLD, "ref_known_answers.json")))
CONFIG_HASH = json.load(open(os.path.join(GOLD, "config_hash.json")))


def test_seed_seq():
    assert list(O.seed_seq([1337], 2)) == KA["seed_seq_1337"] == [2150097757, 2293033019]


def test_pcg32_stream():
    L = O.lib()
    r = O.pcg32(1337)
    assert L.orc_pcg32_next_uint(O.ctypes.byref(r)) == KA["pcg32_1337_next_uint"]
    assert np.float32(L.orc_pcg32_next_float(O.ctypes.byref(r))) == np.float32(KA["pcg32_1337_next_float"])
    r = O.pcg32(1337)
    L.orc_pcg32_advance(O.ctypes.byref(r), 1000003)
    assert L.orc_pcg32_next_uint(O.ctypes.byref(r)) == KA["pcg32_1337_advance_1000003_next_uint"]


def _ends(v, k):
    return np.concatenate([v[:k], v[-k:]])


def test_trainer_init_matches_reference_rng():
    m = O.OracleModel(CONFIG_HASH, 2, 3)
    w = m.w32
    assert m.n_mlp_params == 64 * 32 + 64 * 64 + 16 * 64 == 7168
    assert m.n_params == 7168 + 708368
    w0, w1, wo = w[:2048], w[2048:2048 + 4096], w[6144:7168]
    np.testing.assert_array_equal(_ends(w0, 16), np.float32(KA["xavier_w0_ends16"]))
    np.testing.assert_array_equal(_ends(w1, 16), np.float32(KA["xavier_w1_ends16"]))
    np.testing.assert_array_equal(_ends(wo, 16), np.float32(KA["xavier_wout_ends16"]))
    grid = w[7168:]
    np.testing.assert_array_equal(_ends(grid, 64), np.float32(KA["grid_init_ends64"]))
    assert abs(float(np.sum(grid.astype(np.float64))) - KA["grid_init_sum"]) < 1e-12


def test_batch_rng_strided_order():
    r = O.pcg32(1337)
    b = O.generate_uniform(r, 1 << 19)
    np.testing.assert_array_equal(_ends(b, 64), np.float32(KA["batch_2p19_ends64"]))
    assert O.lib().orc_pcg32_next_uint(O.ctypes.byref(r)) == KA["batch_rng_after_next_uint"]


def test_grid_offset_table_config_hash():
    g = O.grid_cfg(CONFIG_HASH["encoding"], 2)
    sizes = [g.offsets[l + 1] - g.offsets[l] for l in range(16)]
    assert sizes == [256, 576, 1296, 2920, 6568, 14888] + [32768] * 10
    assert g.n_params == 708368
    for l, (sc, res) in enumerate(KA["grid_levels_s1_5"]):
        assert np.float32(g.scales[l]) == np.float32(sc) and g.res[l] == res


def test_grid_offset_table_log2t19():
    enc = dict(CONFIG_HASH["encoding"], log2_hashmap_size=19, per_level_scale=2.0)
    g = O.grid_cfg(enc, 2)
    for l, (sc, res) in enumerate(KA["grid_levels_s2_0"]):
        assert np.float32(g.scales[l]) == np.float32(sc) and g.res[l] == res
    assert g.n_params == 11184640


def test_survey_helper_known_answers():
    # grid_scale(6, log2 1.5, 16) = 181.249985 (res 183),
    # coherent_prime_hash<2>({183,7}) = 1401181024, grid_index<2,CoherentPrime>(Hash, 32768, 183, {183,7}) = 21344
    g = O.grid_cfg(CONFIG_HASH["encoding"], 2)
    assert np.float32(g.scales[6]) == np.float32(181.249985) and g.res[6] == 183
    pg = np.array([183, 7], dtype=np.uint32)
    assert O.lib().orc_coherent_prime_hash(2, O._p(pg)) == 1401181024
    assert O.lib().orc_grid_index(O.ctypes.byref(g), 6, O._p(pg)) == 21344
    # pos_fract(0.3, scale_6) -> pos 0.874996185, grid 54 (fmaf(scale, x, 0.5))
    p = np.float32(np.float64(np.float32(g.scales[6])) * np.float64(np.float32(0.3)) + 0.5)  # exact product, one rounding = fmaf
    assert int(np.floor(p)) == 54 and np.float32(p - np.floor(p)) == np.float32(0.874996185)


def test_fp16_roundtrip_and_rne():
    x = np.array([0.0, -0.0, 1.0, 65504.0, 65520.0, 1e-8, 5.960464477539063e-08, 2.98e-8,
                  3.0e-8, 6.1e-5, 0.333333, -2.5e-6, np.inf, -np.inf], dtype=np.float32)
    h = O.f2h(x)
    ref = x.astype(np.float16).view(np.uint16)
    np.testing.assert_array_equal(h, ref)
    rng = np.random.default_rng(0)
    y = (rng.standard_normal(200000) * np.exp(rng.uniform(-20, 12, 200000))).astype(np.float32)
    np.testing.assert_array_equal(O.f2h(y), y.astype(np.float16).view(np.uint16))
    hh = np.arange(0, 65536, dtype=np.uint32).astype(np.uint16)
    finite = (hh & 0x7c00) != 0x7c00
    np.testing.assert_array_equal(O.h2f(hh[finite]), hh[finite].view(np.float16).astype(np.float32))


def test_hfma_single_rounding():
    rng = np.random.default_rng(1)
    a = rng.uniform(0, 1, 5000).astype(np.float16)
    b = (rng.standard_normal(5000) * 1e-3).astype(np.float16)
    c = (rng.standard_normal(5000) * 1e-3).astype(np.float16)
    L = O.lib()
    for i in range(5000):
        got = L.orc_hfma(int(a[i].view(np.uint16)), int(b[i].view(np.uint16)), int(c[i].view(np.uint16)))
        exact = np.float64(a[i]) * np.float64(b[i]) + np.float64(c[i])
        assert got == np.float16(exact).view(np.uint16), i


# ---- OneBlob restatement (oneblob.h:46-164, common_device.h:905-920) ----
def test_oneblob_partition_of_unity_small_bins():
    """For n_bins <= 32 the reference's shuffle wraps inside the n_bins segment, so the bins of one
    dimension telescope to exactly right(last) - left(0) = 1 (quartic CDF, wrap-around)."""
    rng = np.random.default_rng(0)
    x = rng.random((2000, 2), dtype=np.float32)
    for nb in (4, 16, 32):
        e = O.h2f(O.oneblob_fwd(x, nb)).reshape(2000, 2, nb).astype(np.float64)
        np.testing.assert_allclose(e.sum(axis=2), 1.0, atol=nb * 5e-4)
        assert e.min() >= -1e-3
        # the blob sits on the bin containing x
        peak = e.argmax(axis=2)
        ok = np.abs(((peak + 0.5) / nb - x + 0.5) % 1.0 - 0.5) <= 1.5 / nb
        assert ok.mean() > 0.999


def test_oneblob_64_bins_reproduces_32_lane_shuffle_wrap():
    """n_bins = 64 > warp size: bin 31 reads bin 0's left CDF and bin 63 reads bin 32's
    (+1 wrap), the reference's __shfl_sync(.., bin + 1, 64) semantics on 32-lane warps."""
    x = np.array([[0.3], [0.7], [0.49], [0.99]], np.float32)
    e = O.h2f(O.oneblob_fwd(x, 64))
    assert e[0, 31] == -1.0 and e[0, 63] == 1.0   # x < 0.48: bin 31 = L(0) - L(31) = -1
    assert e[1, 31] == 0.0 and e[1, 63] == 0.0    # 0.5 < x < 0.98
    # bins away from 31/63 are the ordinary quartic blob
    assert abs(e[0, 19] - 0.0) < 1.0 and e[0, 15:24].sum() > 0.99


def test_oneblob_backward_matches_finite_differences():
    rng = np.random.default_rng(1)
    nb = 16
    x = rng.uniform(0.05, 0.95, (64, 2)).astype(np.float32)
    dy = rng.standard_normal((64, 2 * nb)).astype(np.float32)
    dy16 = O.f2h(dy)
    dx = O.oneblob_bwd(x, nb, dy16)
    # reference derivative in float64 from the smooth CDF (no fp16 rounding)
    def L(b, xv):
        def q(t):
            u = t * nb
            return np.clip(15 / 16 * u * (1 - 2 / 3 * u * u + u ** 4 / 5) + 0.5, 0, 1)
        d = b / nb - xv
        return q(d) + q(d - 1) + q(d + 1)
    eps = 1e-4
    dyf = O.h2f(dy16).astype(np.float64).reshape(64, 2, nb)
    fd = np.zeros((64, 2))
    for i in range(64):
        for d in range(2):
            xv = float(x[i, d])
            b = np.arange(nb)
            def enc(v):
                return L(b + 1, v) - L(b, v)
            fd[i, d] = (dyf[i, d] * (enc(xv + eps) - enc(xv - eps)) / (2 * eps)).sum()
    np.testing.assert_allclose(dx, fd, rtol=2e-3, atol=2e-3)


def test_identity_encoding():
    x = np.array([[0.25, -3.0]], np.float32)
    e = O.h2f(O.identity_fwd(x, scale=2.0, offset=0.5, n_pad=2))
    np.testing.assert_array_equal(e, [[1.0, -5.5, 1.0, 1.0]])


def test_grid_input_gradient_matches_analytic_derivative():
    """orc_grid_bwd_input (grid.h:171-211 + 322-349) against a float64 evaluation of d/dx of
    sum_k dL/dy_k * y_k(x) with the same table values and index function (linear interpolation)."""
    enc = dict(CONFIG_HASH["encoding"])
    g = O.grid_cfg(enc, 2)
    rng = np.random.default_rng(3)
    table = O.f2h(rng.uniform(-1, 1, g.n_params).astype(np.float32))
    tf = O.h2f(table).astype(np.float64)
    B = 48
    pos = rng.uniform(0.02, 0.98, (B, 2)).astype(np.float32)
    L, F = g.n_levels, g.n_features_per_level
    dy = O.f2h(rng.standard_normal((L * F, B)).astype(np.float32))
    dyf = O.h2f(dy).astype(np.float64)
    got = O.grid_bwd_input(g, pos, table, dy)
    ref = np.zeros((B, 2))
    pg = np.zeros(2, np.uint32)
    for i in range(B):
        for l in range(L):
            s = np.float32(g.scales[l])
            p = np.float32(s * pos[i] + np.float32(0.5))
            fl = np.floor(p)
            fr = (p - fl).astype(np.float64)
            base = fl.astype(np.int64)
            vals = {}
            for cx in (0, 1):
                for cy in (0, 1):
                    pg[0], pg[1] = base[0] + cx, base[1] + cy
                    idx = O.lib().orc_grid_index(ctypes.byref(g), l, pg.ctypes.data_as(ctypes.c_void_p))
                    vals[(cx, cy)] = tf[(g.offsets[l] + idx) * F:(g.offsets[l] + idx) * F + F]
            dvx = float(s) * ((vals[(1, 0)] - vals[(0, 0)]) * (1 - fr[1]) + (vals[(1, 1)] - vals[(0, 1)]) * fr[1])
            dvy = float(s) * ((vals[(0, 1)] - vals[(0, 0)]) * (1 - fr[0]) + (vals[(1, 1)] - vals[(1, 0)]) * fr[0])
            for f in range(F):
                ref[i, 0] += dyf[l * F + f, i] * dvx[f]
                ref[i, 1] += dyf[l * F + f, i] * dvy[f]
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-3)


def _grid_level_geometry(g, l, x):
    """float64 restatement of one level of the grid for one point: corner table indices and the
    fractional coordinate as a smooth function of x inside the point's cell."""
    s = float(g.scales[l])
    base = np.floor(s * x.astype(np.float64) + 0.5)
    D = len(x)
    idx = []
    pg = np.zeros(D, np.uint32)
    for c in range(1 << D):
        for d in range(D):
            pg[d] = int(base[d]) + ((c >> d) & 1)
        idx.append(O.lib().orc_grid_index(ctypes.byref(g), l, pg.ctypes.data_as(ctypes.c_void_p)))
    return s, base, idx


def _interp(interp, fr):
    if interp == "Smoothstep":
        return fr * fr * (3 - 2 * fr), 6 * fr * (1 - fr)
    return fr, np.ones_like(fr)


def _dydx64(g, interp, l, s, base, idx, x, tf):
    """d y_f / d x_e [F, D] in float64 for the cell given by base."""
    D, F = len(x), g.n_features_per_level
    fr = s * x + 0.5 - base
    p, pd = _interp(interp, fr)
    out = np.zeros((F, D))
    for c in range(1 << D):
        v = tf[(g.offsets[l] + idx[c]) * F:(g.offsets[l] + idx[c]) * F + F]
        for e in range(D):
            w = (1.0 if (c >> e) & 1 else -1.0) * s * pd[e]
            for d in range(D):
                if d != e:
                    w *= p[d] if (c >> d) & 1 else 1 - p[d]
            out[:, e] += w * v
    return out, p, pd


@pytest.mark.parametrize("interp", ["Linear", "Smoothstep"])
def test_grid_second_order_matches_float64_derivatives(interp):
    """orc_grid_bwd_bwd (grid.h:351-627) against float64 derivatives of
    G = sum_{l,f} dL/dy_{l,f} * sum_e dL/d(dL/dx)_e * d y_{l,f} / d x_e:
    dG/dtable analytic, dG/d(dL/dy) analytic, dG/dx by central differences of the analytic dy/dx."""
    enc = dict(CONFIG_HASH["encoding"], interpolation=interp, n_levels=6)
    g = O.grid_cfg(enc, 2)
    rng = np.random.default_rng(11)
    table = O.f2h(rng.uniform(-1, 1, g.n_params).astype(np.float32))
    tf = O.h2f(table).astype(np.float64)
    B, D = 24, 2
    L, F = g.n_levels, g.n_features_per_level
    pos = rng.uniform(0.02, 0.98, (B, D)).astype(np.float32)
    gx = rng.standard_normal((B, D)).astype(np.float32)
    dy = O.f2h(rng.standard_normal((L * F, B)).astype(np.float32))
    dyf = O.h2f(dy).astype(np.float64)
    grad, ddy, dx = O.grid_bwd_bwd(g, pos, table, gx, dy)
    ref_grad = np.zeros(g.n_params)
    ref_ddy = np.zeros((B, L * F))
    ref_dx = np.zeros((B, D))
    h = 1e-9
    for i in range(B):
        x = pos[i].astype(np.float64)
        gi = gx[i].astype(np.float64)
        for l in range(L):
            s, base, idx = _grid_level_geometry(g, l, pos[i])
            J, p, pd = _dydx64(g, interp, l, s, base, idx, x, tf)
            dyl = dyf[l * F:(l + 1) * F, i]
            ref_ddy[i, l * F:(l + 1) * F] = J @ gi
            for c in range(1 << D):
                a = 0.0
                for e in range(D):
                    w = (1.0 if (c >> e) & 1 else -1.0) * s * pd[e] * gi[e]
                    for d in range(D):
                        if d != e:
                            w *= p[d] if (c >> d) & 1 else 1 - p[d]
                    a += w
                o = (g.offsets[l] + idx[c]) * F
                ref_grad[o:o + F] += a * dyl
            for e in range(D):
                xp, xm = x.copy(), x.copy()
                xp[e] += h
                xm[e] -= h
                Jp = _dydx64(g, interp, l, s, base, idx, xp, tf)[0]
                Jm = _dydx64(g, interp, l, s, base, idx, xm, tf)[0]
                ref_dx[i, e] += dyl @ ((Jp - Jm) / (2 * h)) @ gi
    np.testing.assert_allclose(ddy, ref_ddy, rtol=2e-4, atol=2e-4 * np.abs(ref_ddy).max())
    np.testing.assert_allclose(grad, ref_grad, rtol=2e-4, atol=2e-4 * np.abs(ref_grad).max())
    np.testing.assert_allclose(dx, ref_dx, rtol=2e-3, atol=2e-3 * np.abs(ref_dx).max())


def _u2f(u):
    return np.float32(np.uint32((u >> 9) | 0x3F800000).view(np.float32) - np.float32(1.0))


def test_random_val_pinned_to_reference_pcg32():
    """random_val(1337, idx) (common_device.h:333-337) -- the stochastic-interpolation sample --
    against the reference's own pcg32 known answers (oracle/_ref, tests/golden)."""
    assert np.float32(O.random_val(1337, 0)) == _u2f(KA["pcg32_1337_next_uint"])
    assert np.float32(O.random_val(1337, 1)) == np.float32(KA["pcg32_1337_next_float"])
    assert np.float32(O.random_val(1337, 1000003)) == _u2f(KA["pcg32_1337_advance_1000003_next_uint"])


def test_grid_stochastic_backward():
    """kernel_grid_backward with stochastic_interpolation (grid.h:284-298): each (point, level)
    sends its whole dL/dy to the one corner picked by random_val(1337, i + level * B)."""
    enc = dict(CONFIG_HASH["encoding"], n_levels=4, stochastic_interpolation=True)
    g = O.grid_cfg(enc, 2)
    assert g.stochastic == 1
    rng = np.random.default_rng(2)
    B, F, L = 64, g.n_features_per_level, g.n_levels
    pos = rng.uniform(0, 1, (B, 2)).astype(np.float32)
    dy = O.f2h(rng.standard_normal((L * F, B)).astype(np.float32))
    got = O.grid_bwd(g, pos, dy)
    ref = np.zeros(g.n_params, np.float64)
    pg = np.zeros(2, np.uint32)
    for l in range(L):
        s = np.float32(g.scales[l])
        for i in range(B):
            sample = np.float32(O.random_val(1337, i + l * B))
            for d in range(2):
                p = np.float32(np.float64(s) * pos[i, d] + 0.5)  # = fmaf(scale, x, 0.5): one rounding
                fl = np.floor(p)
                pg[d] = int(fl) + (0 if sample >= np.float32(p - fl) else 1)
            idx = O.lib().orc_grid_index(ctypes.byref(g), l, pg.ctypes.data_as(ctypes.c_void_p))
            o = (g.offsets[l] + idx) * F
            ref[o:o + F] += O.h2f(dy[l * F:(l + 1) * F, i])
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-6)


def test_grid_max_level_masking():
    """max_level (grid_interface.h:101-123): levels >= max_level * n_levels (+1e-3) output 0 and
    receive no gradient (grid.h:69-91, 236-244); scalar and per-point variants."""
    enc = dict(CONFIG_HASH["encoding"])
    rng = np.random.default_rng(4)
    g0 = O.grid_cfg(enc, 2)
    table = O.f2h(rng.uniform(-1, 1, g0.n_params).astype(np.float32))
    B, F, L = 256, g0.n_features_per_level, g0.n_levels
    pos = rng.uniform(0, 1, (B, 2)).astype(np.float32)
    full = O.grid_fwd(g0, pos, table)
    g = O.grid_cfg(enc, 2)
    O.grid_set_max_level(g, 0.5)  # 8 levels
    half = O.grid_fwd(g, pos, table)
    np.testing.assert_array_equal(half[:9 * F], full[:9 * F])  # level 8 itself stays (8 >= 8.001 is false)
    assert np.all(half[9 * F:] == 0)
    per_point = rng.uniform(0, 1, B).astype(np.float32)
    gp = O.grid_cfg(enc, 2)
    O.grid_set_max_level(gp, 0.0, per_point)
    pp = O.grid_fwd(gp, pos, table)
    for i in range(B):
        lim = (np.float32(per_point[i]) * np.float32(L * F)) / np.float32(F) + np.float32(1e-3)
        for l in range(L):
            exp = 0 if np.float32(l) >= lim else full[l * F:(l + 1) * F, i]
            np.testing.assert_array_equal(pp[l * F:(l + 1) * F, i], exp)
    dy = O.f2h(rng.standard_normal((L * F, B)).astype(np.float32))
    gb = O.grid_bwd(g, pos, dy)
    gfull = O.grid_bwd(g0, pos, dy)
    cut = g0.offsets[9] * F
    np.testing.assert_array_equal(gb[:cut], gfull[:cut])
    assert np.all(gb[cut:] == 0)


def test_mlp_without_hidden_layers_and_wide_shapes():
    """The restatement's MLP at the shapes the wide layer kernels serve: no hidden layer (CutlassMLP,
    cutlass_mlp.cu:64-67: one [padded_out][in] matrix), W 256 / IN 256 / padded output 144, against a
    float64 evaluation of the same fp16-stored layers (fp16 rounding after every layer, fp32 sums)."""
    rng = np.random.default_rng(7)
    for W, IN, NH, OUTP in ((64, 128, 0, 16), (256, 32, 2, 16), (64, 256, 1, 144)):
        n = O.mlp_n_params(W, IN, NH, OUTP)
        assert n == (OUTP * IN if NH == 0 else W * IN + (NH - 1) * W * W + OUTP * W)
        p16 = O.f2h((rng.standard_normal(n) * 0.1).astype(np.float32))
        B = 64
        x16 = O.f2h(rng.random((B, IN), dtype=np.float32))
        out, hidden = O.mlp_fwd(W, IN, NH, OUTP, p16, x16, input_soa=False, activation=1)
        pf = O.h2f(p16).astype(np.float64)
        a = O.h2f(x16).astype(np.float64)
        off, k, acts = 0, IN, [a]
        for _ in range(NH):
            Wm = pf[off:off + W * k].reshape(W, k)
            off += W * k
            a = np.maximum(a @ Wm.T, 0).astype(np.float16).astype(np.float64)
            acts.append(a)
            k = W
        Wo = pf[off:off + OUTP * k].reshape(OUTP, k)
        ref = a @ Wo.T
        np.testing.assert_allclose(O.h2f(out).astype(np.float64), ref, rtol=2e-3, atol=2e-3 * np.abs(ref).max())
        dout = O.f2h((rng.standard_normal((B, OUTP)) * 0.01).astype(np.float32))
        wg, din = O.mlp_bwd(W, IN, NH, OUTP, p16, x16, hidden, dout, input_soa=False, activation=1)
        g = O.h2f(dout).astype(np.float64)
        np.testing.assert_allclose(wg[off:], (g.T @ acts[-1]).ravel(), rtol=1e-4, atol=1e-6)
        if NH == 0:
            np.testing.assert_allclose(O.h2f(din), g @ Wo, rtol=2e-3, atol=1e-5)
