"""GPU tests of the smaller reference API surface:
  * L2Loss (losses/l2.h:40-76) on the fused and the layer-wise engine, against the oracle
    (loss sum rel 1e-3, gradient vectors rel-L2 1e-3 -- the parity bar of test_gpu_parity.py)
  * torch modules pickle / unpickle (modules.py:194-204) and expose n_output_dims() / n_params() as
    methods on the native module (bindings.cpp, modules.py:326)
  * tcnn::cpp::set_log_callback (cpp_api.cu:61-63) receives the engine's debug messages
  * Trainer::deserialize of the JSON form of a snapshot, binaries as {"bytes": [...]}
    (gpu_memory_json.h:58-67)
"""
import copy
import ctypes
import io
import json
import pickle

import numpy as np
import pytest

from helpers import CONFIG_HASH, CONFIG_ONEBLOB, make_batch, rel_err, trainer_arrays
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available()
    return torch


def _l2_config(base):
    cfg = copy.deepcopy(base)
    cfg["loss"] = {"otype": "L2"}
    return cfg


@pytest.mark.parametrize("which", ["fused", "tile", "layered"])
def test_l2_loss_step_matches_oracle(torch_mod, which):
    torch = torch_mod
    from tinycudann import Trainer
    if which == "fused":
        cfg = _l2_config(CONFIG_HASH)
    else:
        cfg = _l2_config(CONFIG_ONEBLOB)
        cfg["network"] = dict(cfg["network"], n_neurons=64, n_hidden_layers=2)
        if which == "layered":
            cfg["network"]["otype"] = "CutlassMLP"
    t = Trainer(2, 3, cfg, seed=1337)
    assert t.engine == ("layered" if which == "layered" else "fused")
    om = O.OracleModel(cfg, 2, 3, seed=1337)
    B = 2048
    pos, tgt = make_batch(B)
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    loss_gpu = t.loss()
    loss_ref = om.train_step(pos, tgt, run_optimizer=False)
    # the L2 sum is not the RelativeL2 one (pins that the loss kind reached the kernel)
    assert abs(loss_gpu - loss_ref) <= 1e-3 * abs(loss_ref), (loss_gpu, loss_ref)
    a = trainer_arrays(t)
    nm = om.n_mlp_params
    assert rel_err(a["g32"][:nm], om.grad32[:nm]) <= 1e-3
    if om.n_params > nm:
        assert rel_err(a["g32"][nm:], om.grad32[nm:]) <= 1e-3
    # a few optimiser steps keep tracking the oracle
    for s in range(1, 5):
        pos, tgt = make_batch(B, step=s)
        t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda())
        lg = t.loss()
        lr = om.train_step(pos, tgt, n_threads=4)
        assert abs(lg - lr) <= 3e-2 * abs(lr), (s, lg, lr)


def test_l2_loss_values_kernel_vs_oracle_relative(torch_mod):
    """Both losses on the same prediction: L2 != RelativeL2 (guards against a silently ignored otype)."""
    torch = torch_mod
    from tinycudann import Trainer
    pos, tgt = make_batch(1024)
    losses = {}
    for otype in ("RelativeL2", "L2"):
        cfg = copy.deepcopy(CONFIG_HASH)
        cfg["loss"] = {"otype": otype}
        t = Trainer(2, 3, cfg, seed=1337)
        t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
        losses[otype] = t.loss()
    assert abs(losses["L2"] - losses["RelativeL2"]) > 1e-3 * losses["L2"], losses


def test_unknown_loss_rejected(torch_mod):
    from tinycudann import Trainer
    from tinycudann._lib import TcnnError
    cfg = copy.deepcopy(CONFIG_HASH)
    cfg["loss"] = {"otype": "Huber"}
    with pytest.raises(TcnnError):
        Trainer(2, 3, cfg, seed=1337)


def test_modules_pickle_roundtrip(torch_mod):
    torch = torch_mod
    import tinycudann as tcnn
    m = tcnn.NetworkWithInputEncoding(2, 3, CONFIG_HASH["encoding"], CONFIG_HASH["network"], seed=7)
    x = torch.rand(1000, 2, device="cuda")
    with torch.no_grad():
        y0 = m(x).float()
    buf = io.BytesIO()
    torch.save(m, buf)
    buf.seek(0)
    m2 = torch.load(buf, weights_only=False)  # our own object, written just above
    with torch.no_grad():
        y1 = m2(x).float()
    torch.testing.assert_close(y0, y1, rtol=0, atol=0)
    e = tcnn.Encoding(2, CONFIG_HASH["encoding"])
    e2 = pickle.loads(pickle.dumps(e))
    assert e2.n_output_dims == e.n_output_dims == 32
    with torch.no_grad():
        torch.testing.assert_close(e(x), e2(x), rtol=0, atol=0)


def test_native_module_sizes_are_methods(torch_mod):
    import tinycudann as tcnn
    e = tcnn.Encoding(2, CONFIG_HASH["encoding"])
    nm = e.native_tcnn_module
    assert nm.n_input_dims() == 2 and nm.n_output_dims() == 32
    assert nm.n_params() == 708368
    n = tcnn.Network(32, 3, CONFIG_HASH["network"])
    assert n.native_tcnn_module.n_output_dims() == 16  # padded width (cpp_api.cu:130)


def test_log_callback_receives_engine_messages(torch_mod):
    from tinycudann import _lib as L
    lib = L.lib()
    got = []
    cb = L.LOG_CALLBACK(lambda sev, msg, user: got.append((sev, msg.decode())))
    lib.tcnn_set_log_callback(cb, None)
    try:
        from tinycudann import Trainer
        Trainer(2, 3, CONFIG_HASH, seed=1337)
    finally:
        lib.tcnn_set_log_callback(L.LOG_CALLBACK(), None)  # NULL: remove
    msgs = [m for _, m in got]
    assert any(m.startswith("GridEncoding at level 6: resolution=183") for m in msgs), msgs[:8]
    assert any("Trainer: initializing 715536 params" in m for m in msgs)
    assert all(sev == 1 for sev, _ in got)  # Debug


def test_deserialize_json_object_binaries(torch_mod):
    torch = torch_mod
    from tinycudann import Trainer
    cfg = copy.deepcopy(CONFIG_ONEBLOB)  # small parameter vector: the JSON form is ~10 bytes per byte
    cfg["network"] = dict(cfg["network"], n_neurons=64, n_hidden_layers=2)
    ta = Trainer(2, 3, cfg, seed=1337)
    pos, tgt = make_batch(1024)
    ta.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda())
    import msgpack
    snap = msgpack.unpackb(ta.serialize(optimizer=True), raw=False)

    def to_json(v):
        if isinstance(v, (bytes, bytearray)):
            return {"bytes": list(v), "subtype": None}
        if isinstance(v, dict):
            return {k: to_json(x) for k, x in v.items()}
        return v

    text = json.dumps(to_json(snap)).encode()
    tb = Trainer(2, 3, cfg, seed=99)
    tb.deserialize(text)
    a, b = trainer_arrays(ta), trainer_arrays(tb)
    np.testing.assert_array_equal(a["w16"], b["w16"])
    assert tb.optimizer_step_count == ta.optimizer_step_count == 1
