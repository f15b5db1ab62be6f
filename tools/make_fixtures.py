"""Generate the SURVEY Appendix C fixtures F3-F7 from the CPU oracle (oracle/, test infrastructure)
and freeze them under tests/golden/. Inputs are regenerated from pcg32 seeds (oracle.generate_uniform,
the reference's generate_random_uniform order), so only outputs are stored.

  F3 f3_grid_fwd.npz      kernel_grid (grid.h:48-212): config_hash grid, B=4096, table = 5000 x the
                          seed-1337 init (O(1) values exercise the fp16 FMA chain); enc fp16 [32][B]
  F4 f4_grid_bwd.npz      kernel_grid_backward (grid.h:214-320): B=1024, fixed dL/dy; the touched
                          gradient entries (sparse index + fp32 value) and their per-element bound
  F5 f5_mlp_*.npz         FullyFusedMLP fwd / bwd / wgrad (fully_fused_mlp.cu:47-557, 735-836) at
                          B=1024 for (W, H, IN) in (64, 2, 32), (128, 4, 32), (128, 5, 128)
  F6 f6_loss_adam.npz     RelativeL2 + L2 values / gradients (relative_l2.h, l2.h); Adam 1 and 10 steps
                          (adam.h:47-188) on 4096 params, 1/4 of the non-matrix gradients zero
  F7 f7_train20.json      20 Trainer::training_steps of config_hash at B=4096 from seed 1337: per-step
                          loss, final parameter norms

The CPU suite (tests/test_fixtures.py) checks that the live oracle still reproduces every fixture
bit for bit, and that an independent float64 numpy restatement agrees with F3 / F5; the GPU suite
(tests/test_gpu_fixtures.py) checks the HIP path against the frozen vectors.

usage: python tools/make_fixtures.py
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from oracle import oracle as O  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden")
CONFIG_HASH = json.load(open(os.path.join(GOLD, "config_hash.json")))
MLP_SHAPES = [(64, 2, 32), (128, 4, 32), (128, 5, 128)]


def uniform(seed, n, lo=0.0, hi=1.0):
    return O.generate_uniform(O.pcg32(seed), n, lo, hi)


def f3_inputs():
    g = O.grid_cfg(CONFIG_HASH["encoding"], 2)
    pos = uniform(1337, 2 * 4096).reshape(4096, 2)
    table = O.f2h(uniform(7, g.n_params, -1e-4, 1e-4) * 5000.0)
    return g, pos, table


def f4_inputs():
    g = O.grid_cfg(CONFIG_HASH["encoding"], 2)
    B = 1024
    pos = uniform(11, 2 * B).reshape(B, 2)
    dy = O.f2h(uniform(12, g.n_levels * g.n_features_per_level * B, -1.0, 1.0)).reshape(-1, B)  # SoA [L*F][B]
    return g, pos, dy


def f5_inputs(W, H, IN):
    B = 1024
    n = O.mlp_n_params(W, IN, H, 16)
    params = O.f2h(uniform(100 + W + H, n, -1.0, 1.0) * np.float32(np.sqrt(6.0 / (W + W))))
    x = O.f2h(uniform(200 + IN, IN * B, -1.0, 1.0)).reshape(B, IN)  # AoS [B][IN]
    dout = O.f2h(uniform(300 + W, 16 * B, -1.0, 1.0)).reshape(B, 16)  # loss-scaled magnitudes (x128)
    return params, x, dout


def f6_inputs():
    B = 1024
    pred = O.f2h(uniform(400, 16 * B, -0.5, 1.5)).reshape(B, 16)
    target = uniform(401, 3 * B).reshape(B, 3)
    n, n_matrix = 4096, 3072
    w32 = uniform(402, n, -0.1, 0.1)
    grads = [O.f2h(uniform(410 + s, n, -128.0, 128.0)) for s in range(10)]
    for s, gr in enumerate(grads):  # a quarter of the non-matrix gradients are zero each step
        gr[n_matrix + (np.arange(n - n_matrix) % 4 == s % 4).nonzero()[0]] = 0
    return pred, target, w32, grads, n_matrix


def f7_batch(step, B=4096):
    import helpers
    return helpers.make_batch(B, step=step)


def compute_all():
    out = {}
    g, pos, table = f3_inputs()
    out["f3_grid_fwd"] = {"enc": O.grid_fwd(g, pos, table)}

    g, pos, dy = f4_inputs()
    grad = O.grid_bwd(g, pos, dy)
    idx = np.nonzero(grad)[0].astype(np.uint32)
    tol = O.grid_grad_tolerance(g, pos, dy, grad)
    out["f4_grid_bwd"] = {"idx": idx, "val": grad[idx], "tol": tol[idx].astype(np.float32), "n_params": np.array([g.n_params])}

    for W, H, IN in MLP_SHAPES:
        params, x, dout = f5_inputs(W, H, IN)
        y, hidden = O.mlp_fwd(W, IN, H, 16, params, x, input_soa=False)
        wg, din = O.mlp_bwd(W, IN, H, 16, params, x, hidden, dout, input_soa=False)
        out[f"f5_mlp_w{W}_h{H}_in{IN}"] = {"out": y, "wgrad": wg, "dinput": din}

    pred, target, w32, grads, n_matrix = f6_inputs()
    s_rel, g_rel, v_rel = O.relative_l2(pred, target, want_values=True)
    s_l2, g_l2, v_l2 = O.l2(pred, target, want_values=True)
    cfg = O.adam_cfg({"learning_rate": 1e-2, "beta1": 0.9, "beta2": 0.99, "l2_reg": 1e-6})
    res = {"rel_sum": np.array([s_rel]), "rel_grad": g_rel, "rel_val": v_rel, "l2_sum": np.array([s_l2]), "l2_grad": g_l2,
           "l2_val": v_l2}
    w, w16 = w32.copy(), O.f2h(w32)
    m1 = np.zeros_like(w)
    m2 = np.zeros_like(w)
    steps = np.zeros(len(w), np.uint32)
    for s in range(10):
        O.adam_step(cfg, n_matrix, 128.0, s + 1, w, w16, grads[s], m1, m2, steps)
        if s == 0:
            res["adam1_w32"] = w.copy()
    res.update({"adam10_w32": w, "adam10_w16": w16, "adam10_m1": m1, "adam10_m2": m2, "adam10_steps": steps})
    out["f6_loss_adam"] = res

    om = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
    losses = [float(om.train_step(*f7_batch(s), n_threads=4)) for s in range(20)]
    nm = om.n_mlp_params
    out["f7_train20"] = {"loss": losses, "mlp_l2": float(np.linalg.norm(om.w32[:nm].astype(np.float64))),
                         "grid_l2": float(np.linalg.norm(om.w32[nm:].astype(np.float64)))}
    return out


def main():
    out = compute_all()
    for name, d in out.items():
        if name == "f7_train20":
            with open(os.path.join(GOLD, name + ".json"), "w") as f:
                json.dump(d, f, indent=1)
        else:
            np.savez_compressed(os.path.join(GOLD, name + ".npz"), **d)
        p = os.path.join(GOLD, name + (".json" if name == "f7_train20" else ".npz"))
        print(f"{p}: {os.path.getsize(p)} bytes")


if __name__ == "__main__":
    main()
