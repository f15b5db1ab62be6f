"""Trainer snapshots in the reference's format (Trainer::serialize /
deserialize, trainer.h:275-315; Adam state adam.h:278-299; binary blobs gpu_memory_json.h:36-71),
written as json::to_msgpack would. Checked with the independent `msgpack` Python package."""
import msgpack
import numpy as np
import pytest

from helpers import CONFIG_HASH, CONFIG_ONEBLOB, make_batch, rel_err, trainer_arrays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available()
    return torch


def _steps(torch, t, n, B=2048, start=0):
    for s in range(start, start + n):
        pos, tgt = make_batch(B, step=s)
        t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda())
        t.loss()


def test_snapshot_layout_matches_reference_schema(torch_mod):
    torch = torch_mod
    from tinycudann import Trainer
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    _steps(torch, t, 3)
    a = trainer_arrays(t)
    d = msgpack.unpackb(t.serialize(optimizer=True), raw=False)
    assert sorted(d) == ["n_params", "optimizer", "params_binary", "params_type"]
    assert d["n_params"] == t.n_params and d["params_type"] == "__half"
    np.testing.assert_array_equal(np.frombuffer(d["params_binary"], np.uint16), a["w16"])
    o = d["optimizer"]
    assert sorted(o) == ["base_learning_rate", "current_step", "first_moments_binary", "param_steps_binary",
                         "second_moments_binary"]
    assert o["current_step"] == 3 and abs(o["base_learning_rate"] - 1e-2) < 1e-9
    assert len(o["first_moments_binary"]) == 4 * t.n_params
    steps = np.frombuffer(o["param_steps_binary"], np.uint32)
    assert steps.max() == 3
    d2 = msgpack.unpackb(t.serialize(optimizer=False), raw=False)
    assert "optimizer" not in d2


@pytest.mark.parametrize("cfg", [CONFIG_HASH, CONFIG_ONEBLOB], ids=["hash", "oneblob"])
def test_snapshot_roundtrip_resumes_training(torch_mod, cfg):
    """deserialize(serialize(A)) into a differently seeded trainer B: identical fp16 params and Adam
    state, identical next-step loss (the forward reads the fp16 params); the fp32 master becomes
    (float)half as in the reference (trainer.h:295-304), so later parameters agree to fp16 ulps."""
    torch = torch_mod
    from tinycudann import Trainer
    ta = Trainer(2, 3, cfg, seed=1337)
    _steps(torch, ta, 4)
    blob = ta.serialize(optimizer=True)
    tb = Trainer(2, 3, cfg, seed=7)
    tb.deserialize(blob)
    a, b = trainer_arrays(ta), trainer_arrays(tb)
    np.testing.assert_array_equal(a["w16"], b["w16"])
    np.testing.assert_array_equal(b["w32"], a["w16"].view(np.float16).astype(np.float32))
    assert tb.optimizer_step_count == ta.optimizer_step_count == 4
    pos, tgt = make_batch(2048, step=4)
    for t in (ta, tb):
        t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda())
    assert ta.loss() == tb.loss()
    a, b = trainer_arrays(ta), trainer_arrays(tb)
    assert rel_err(b["w32"], a["w32"]) < 1e-3


def test_snapshot_accepts_reference_written_blob(torch_mod):
    """A snapshot packed by a different msgpack writer (the `msgpack` package, fp32 params as
    params_type "float", float64 learning rate, no param_steps) deserializes."""
    torch = torch_mod
    from tinycudann import Trainer
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    n = t.n_params
    rng = np.random.default_rng(0)
    w = rng.uniform(-0.1, 0.1, n).astype(np.float32)
    m1 = rng.standard_normal(n).astype(np.float32)
    m2 = rng.uniform(0, 1, n).astype(np.float32)
    blob = msgpack.packb({"n_params": n, "params_type": "float", "params_binary": w.tobytes(),
                          "optimizer": {"current_step": 17, "base_learning_rate": 0.005,
                                        "first_moments_binary": m1.tobytes(), "second_moments_binary": m2.tobytes()}},
                         use_bin_type=True)
    t.deserialize(blob)
    a = trainer_arrays(t)
    np.testing.assert_array_equal(a["w32"], w)
    np.testing.assert_array_equal(a["w16"], w.astype(np.float16).view(np.uint16))
    assert t.optimizer_step_count == 17
    with pytest.raises(Exception):
        t.deserialize(blob[:-10])  # truncated
