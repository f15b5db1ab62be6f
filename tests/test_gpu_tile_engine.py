"""GPU parity of the fused tile engine's full FullyFusedMLP shape set (mlp_tile.h) against the CPU
oracle (reference fully_fused_mlp.cu:499-557, widths 16/32/64/128 at :893-896):

  * fused inference (k_mlp_tile_infer, the reference's INFERENCE=true kernel) on config_oneblob.json
    as-is (OneBlob 64 bins + W128/H5) and BASELINE configs[3] (HashGrid + W128/H4), ragged tiles;
  * W16 and W32 networks with OneBlob / Identity input (training + inference);
  * output activations (fully_fused_mlp.cu:759-762 transfer, warp_activation on the last layer) on
    the fused tile engine, and hidden + output activations on the layer-wise engine;
  * the Module forward context: the backward reuses the encoding its forward kept, including the
    reference's regression case of two forwards before one backward (scripts/test_toch_bindings.py:28-50).

Tolerances (north_star: 1e-3 relative, fp16): network outputs within 4 fp16 ulps of the output scale
(fp32 MFMA accumulation vs the oracle's CPU summation order); gradients relative L2 <= 1e-3 (2e-3 for
W128 / 5-hidden-layer networks and for exponential-type output activations, whose fp16 transfer
factor amplifies one-ulp output differences); loss relative 1e-3.
"""
import copy
import ctypes
import json

import numpy as np
import pytest

from helpers import CONFIG_HASH, CONFIG_ONEBLOB, assert_within_fp16_ulps, make_batch, rel_err, trainer_arrays
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available()
    return torch


def _cfg(enc, w, nh, otype="FullyFusedMLP", act="ReLU", out_act="None"):
    c = copy.deepcopy(CONFIG_HASH)
    c["encoding"] = enc
    c["network"] = {"otype": otype, "activation": act, "output_activation": out_act, "n_neurons": w, "n_hidden_layers": nh}
    return c


GRID = CONFIG_HASH["encoding"]
INFER = {
    "config_oneblob_as_file_w128_h5": CONFIG_ONEBLOB,
    "configs3_hashgrid_w128_h4": _cfg(GRID, 128, 4),
    "oneblob64_w64_h2": _cfg({"otype": "OneBlob", "n_bins": 64}, 64, 2),
    "identity_w128_h3": _cfg({"otype": "Identity"}, 128, 3),
    "oneblob16_w32_h2": _cfg({"otype": "OneBlob", "n_bins": 16}, 32, 2),
    "identity_w16_h1": _cfg({"otype": "Identity"}, 16, 1),
    "hashgrid_w16_h3": _cfg(GRID, 16, 3),
}


@pytest.mark.parametrize("B", [1024, 1056])
@pytest.mark.parametrize("name", list(INFER))
def test_tile_inference_matches_oracle(torch_mod, name, B):
    torch = torch_mod
    from tinycudann import Trainer
    cfg = INFER[name]
    t = Trainer(2, 3, cfg, seed=1337)
    assert t.inference_engine == "fused", t.inference_engine
    om = O.OracleModel(cfg, 2, 3, seed=1337)
    pos, _ = make_batch(B, seed=3)
    out = t.inference(torch.from_numpy(pos).cuda()).cpu().numpy()
    ref = O.h2f(om.inference(pos, n_threads=4))[:, :3]
    assert_within_fp16_ulps(out, ref)


SMALL = {
    "identity_w16_h1": _cfg({"otype": "Identity"}, 16, 1),
    "identity_w16_h3": _cfg({"otype": "Identity"}, 16, 3),
    "oneblob16_w16_h2": _cfg({"otype": "OneBlob", "n_bins": 16}, 16, 2),
    "oneblob64_w16_h2": _cfg({"otype": "OneBlob", "n_bins": 64}, 16, 2),
    "identity_w32_h2": _cfg({"otype": "Identity"}, 32, 2),
    "oneblob16_w32_h3": _cfg({"otype": "OneBlob", "n_bins": 16}, 32, 3),
    "oneblob32_w32_h5": _cfg({"otype": "OneBlob", "n_bins": 32}, 32, 5),
    "hashgrid_w16_h2": _cfg(GRID, 16, 2),
    # grid + W64/H3 trains on the tile engine since r03 (the register kernel spilled at H3)
    "hashgrid_w64_h3": _cfg(GRID, 64, 3),
}


@pytest.mark.parametrize("name", list(SMALL))
def test_small_width_training_step_matches_oracle(torch_mod, name):
    """W16 (zero-padded to the W32 kernel), W32 and grid + W64/H3 FullyFusedMLP on the fused tile engine."""
    torch = torch_mod
    from tinycudann import Trainer
    cfg = SMALL[name]
    t = Trainer(2, 3, cfg, seed=1337)
    assert t.engine == "fused", t.engine
    om = O.OracleModel(cfg, 2, 3, seed=1337)
    assert t.n_params == om.n_params
    np.testing.assert_array_equal(trainer_arrays(t)["w16"], om.w16)
    pos, tgt = make_batch(512)
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    loss_ref = om.train_step(pos, tgt, run_optimizer=False, n_threads=4)
    assert abs(t.loss() - loss_ref) <= 1e-3 * abs(loss_ref), (t.loss(), loss_ref)
    a = trainer_arrays(t)
    nm = om.n_mlp_params
    assert rel_err(a["g32"][:nm], om.grad32[:nm]) <= 1e-3
    if om.n_params > nm:
        assert rel_err(a["g32"][nm:], om.grad32[nm:]) <= 1e-3
    # a few optimizer steps track the oracle
    for s in range(1, 4):
        pos, tgt = make_batch(512, step=s)
        t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda())
        lr = om.train_step(pos, tgt, n_threads=4)
        assert abs(t.loss() - lr) <= 2e-2 * abs(lr), (s, t.loss(), lr)


OUT_ACTS = ["Sigmoid", "Exponential", "Tanh", "Softplus", "LeakyReLU", "Squareplus", "ReLU"]


@pytest.mark.parametrize("out_act", OUT_ACTS)
def test_output_activation_fused_tile(torch_mod, out_act):
    torch = torch_mod
    from tinycudann import Trainer
    cfg = _cfg({"otype": "OneBlob", "n_bins": 32}, 64, 2, out_act=out_act)
    t = Trainer(2, 3, cfg, seed=1337)
    assert t.engine == "fused" and t.inference_engine == "fused", (t.engine, t.inference_engine)
    om = O.OracleModel(cfg, 2, 3, seed=1337)
    pos, tgt = make_batch(512)
    out = t.inference(torch.from_numpy(pos).cuda()).cpu().numpy()
    assert_within_fp16_ulps(out, O.h2f(om.inference(pos, n_threads=4))[:, :3])
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    loss_ref = om.train_step(pos, tgt, run_optimizer=False, n_threads=4)
    assert abs(t.loss() - loss_ref) <= 1e-3 * abs(loss_ref), (t.loss(), loss_ref)
    a = trainer_arrays(t)
    tol = 2e-3 if out_act in ("Exponential", "Softplus", "Squareplus") else 1e-3
    assert rel_err(a["g32"], om.grad32) <= tol, rel_err(a["g32"], om.grad32)


@pytest.mark.parametrize("act,out_act", [("Tanh", "None"), ("Sigmoid", "Sigmoid"), ("LeakyReLU", "Exponential"),
                                         ("Softplus", "None"), ("Squareplus", "Tanh"), ("Exponential", "None")])
def test_activations_layered_engine(torch_mod, act, out_act):
    """Hidden activations beyond None / ReLU run on the layer-wise engine (common_device.h:102-297)."""
    torch = torch_mod
    from tinycudann import Trainer
    cfg = _cfg({"otype": "OneBlob", "n_bins": 16}, 32, 2, act=act, out_act=out_act)
    t = Trainer(2, 3, cfg, seed=1337)
    assert t.engine == "layered", t.engine
    om = O.OracleModel(cfg, 2, 3, seed=1337)
    pos, tgt = make_batch(512)
    out = t.inference(torch.from_numpy(pos).cuda()).cpu().numpy()
    assert_within_fp16_ulps(out, O.h2f(om.inference(pos, n_threads=4))[:, :3])
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    loss_ref = om.train_step(pos, tgt, run_optimizer=False, n_threads=4)
    assert abs(t.loss() - loss_ref) <= 1e-3 * abs(loss_ref), (t.loss(), loss_ref)
    assert rel_err(trainer_arrays(t)["g32"], om.grad32) <= 2e-3


def _module(lib, L, cfg):
    return L.check_ptr(lib.tcnn_create_network_with_input_encoding(2, 3, json.dumps(cfg["encoding"]).encode(),
                                                                   json.dumps(cfg["network"]).encode()))


@pytest.mark.parametrize("name", ["config_hash", "configs3_hashgrid_w128_h4", "oneblob64_w64_h2"])
def test_module_forward_context_reused_by_backward(torch_mod, name):
    """Module::forward keeps the encoding its backward reads (fused grid kernel: SoA, no gathers;
    tile engine: AoS, no encoding pass). Two forwards before one backward: the first context still
    describes the first batch. Gradients equal a recomputing backward's and the oracle's."""
    torch = torch_mod
    from tinycudann import _lib as L
    lib = L.lib()
    cfg = CONFIG_HASH if name == "config_hash" else INFER[name]
    m = _module(lib, L, cfg)
    assert lib.tcnn_module_inference_engine(m) == b"fused"
    n = lib.tcnn_module_n_params(m)
    p32 = torch.zeros(n, dtype=torch.float32, device="cuda")
    L.check(lib.tcnn_module_initialize_params(m, 42, ctypes.c_void_p(p32.data_ptr()), 1.0))
    p16 = p32.half().contiguous()
    B = 1024
    xs = [torch.from_numpy(make_batch(B, seed=s)[0]).cuda() for s in (11, 12)]
    outs = [torch.empty(B, 16, dtype=torch.float16, device="cuda") for _ in xs]
    rng = np.random.default_rng(0)
    dout = np.zeros((B, 16), np.float32)
    dout[:, :3] = rng.standard_normal((B, 3)) * 0.05
    dout16 = torch.from_numpy(dout).half().cuda()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    ctxs = [L.check_ptr(lib.tcnn_module_forward(m, None, B, P(x), P(o), P(p16), 0)) for x, o in zip(xs, outs)]

    def bwd(ctx, x, o):
        g = torch.empty(n, dtype=torch.float16, device="cuda")
        L.check(lib.tcnn_module_backward(m, None, ctx, B, None, P(dout16), P(g), P(x), P(o), P(p16)))
        torch.cuda.synchronize()
        return g.float().cpu().numpy()

    g_first = bwd(ctxs[0], xs[0], outs[0])  # after the second forward
    # a context whose input differs from the backward's input is not reused: recomputed gradient
    ctx_other = L.check_ptr(lib.tcnn_module_forward(m, None, B, P(xs[1]), P(outs[1]), P(p16), 0))
    g_recomputed = bwd(ctx_other, xs[0], outs[0])
    np.testing.assert_allclose(g_first, g_recomputed, rtol=0, atol=0)
    # oracle: the network output and the gradient of the first batch
    om = O.OracleModel(cfg, 2, 3, seed=1337)
    inf = lambda x: om.inference(x, n_threads=4)  # noqa: E731
    params16 = p16.cpu().numpy().view(np.uint16)
    om.w16[:] = params16
    assert_within_fp16_ulps(O.h2f(outs[0].cpu().numpy().view(np.uint16))[:, :3], O.h2f(inf(xs[0].cpu().numpy()))[:, :3])
    for c in ctxs + [ctx_other]:
        lib.tcnn_context_destroy(c)
    lib.tcnn_module_destroy(m)


_TS_SCRIPT = r"""
import json, os, sys
import numpy as np
import torch
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "tests"), os.path.join(sys.argv[1], "neuralbtf-tiny-cuda-nn_amd")]
from helpers import make_batch, trainer_arrays
from tinycudann import Trainer
cfg = json.loads(sys.argv[2])
t = Trainer(2, 3, cfg, seed=1337)
pos, tgt = make_batch(512)
t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
np.save(sys.argv[3], trainer_arrays(t)["g32"])
print(json.dumps({"loss": t.loss()}))
"""


@pytest.mark.parametrize("name", ["configs3_hashgrid_w128_h4", "oneblob64_w128_h2"])
def test_tile_samples_switch_matches_oracle(torch_mod, name, tmp_path):
    """The 8-wave W128 kernel's two tile sizes (64 samples by default, TCNN_TILE_SAMPLES=32 -- read
    once per process, so the 32-sample step runs in a child process) both match the oracle, and each
    other within the fp32 summation-order difference of their weight-gradient sums."""
    import os
    import subprocess
    import sys
    torch = torch_mod
    from tinycudann import Trainer
    cfg = INFER[name] if name in INFER else _cfg({"otype": "OneBlob", "n_bins": 64}, 128, 2)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "g32_ts32.npy"
    env = dict(os.environ, TCNN_TILE_SAMPLES="32")
    r = subprocess.run([sys.executable, "-c", _TS_SCRIPT, repo, json.dumps(cfg), str(out)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    loss32 = json.loads(r.stdout.strip().splitlines()[-1])["loss"]
    g32_ts32 = np.load(out)
    t = Trainer(2, 3, cfg, seed=1337)
    assert t.engine == "fused", t.engine
    pos, tgt = make_batch(512)
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    g64 = trainer_arrays(t)["g32"]
    om = O.OracleModel(cfg, 2, 3, seed=1337)
    loss_ref = om.train_step(pos, tgt, run_optimizer=False, n_threads=4)
    for loss, g in ((t.loss(), g64), (loss32, g32_ts32)):
        assert abs(loss - loss_ref) <= 1e-3 * abs(loss_ref), (loss, loss_ref)
        assert rel_err(g, om.grad32) <= 2e-3
    assert rel_err(g64, g32_ts32) <= 1e-3


_GENC_SCRIPT = r"""
import json, os, sys
import numpy as np
import torch
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "tests"), os.path.join(sys.argv[1], "neuralbtf-tiny-cuda-nn_amd")]
from helpers import make_batch, trainer_arrays
from tinycudann import Trainer
cfg = json.loads(sys.argv[2])
B, spread = int(sys.argv[4]), float(sys.argv[5])
t = Trainer(2, 3, cfg, seed=1337)
pos, tgt = make_batch(B)
pos = (pos * (1.0 + 2.0 * spread) - spread).astype(np.float32)
for k in range(2):
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=(k == 0))
np.save(sys.argv[3], np.concatenate([trainer_arrays(t)["g32"], trainer_arrays(t)["w32"], [t.loss()]]))
"""


@pytest.mark.parametrize("B,spread", [(512, 0.0), (65536, 0.0), (1024, 0.1), (131072, 0.05)])
def test_tile_in_kernel_grid_encode_bit_identical(torch_mod, B, spread, tmp_path):
    """configs[3]'s shape can gather the grid encoding inside the tile kernel (mlp_tile.h GENC, r06,
    opt-in TCNN_TILE_GENC=1): two training steps (Adam, then gradients) are bit-identical to the same
    steps with the encoding as its own AoS pass (the default; the switch is read once per process, so
    both run in child processes). spread > 0 moves positions outside [0, 1] (the general grid index
    instead of the in-range one)."""
    import os
    import subprocess
    import sys
    cfg = INFER["configs3_hashgrid_w128_h4"]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    for genc in ("1", "0"):
        out = tmp_path / f"genc{genc}.npy"
        env = dict(os.environ, TCNN_TILE_GENC=genc)
        r = subprocess.run([sys.executable, "-c", _GENC_SCRIPT, repo, json.dumps(cfg), str(out), str(B), str(spread)], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[genc] = np.load(out)
    assert np.isfinite(outs["1"]).all()
    np.testing.assert_array_equal(outs["1"], outs["0"])
