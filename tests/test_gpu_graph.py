"""hipGraph replay of the training step (the reference Trainer's CUDA graph, trainer.h:163-190,
cuda_graph.h:52-178): a trainer replaying captured graphs must produce bit-identical parameters,
Adam state and losses to an eager trainer over the same steps -- including re-capture after a
hyper-parameter change and after a batch-size change."""
import ctypes
import json

import numpy as np
import pytest

from helpers import CONFIG_HASH, make_batch, trainer_arrays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available()
    return torch


def _update_lr(t, lr):
    from tinycudann import _lib as L
    L.check(L.lib().tcnn_trainer_update_hyperparams(t.h, json.dumps({"optimizer": {"learning_rate": lr}}).encode()))


def test_graph_replay_bit_identical(torch_mod):
    torch = torch_mod
    from tinycudann import Trainer
    eager = Trainer(2, 3, CONFIG_HASH, seed=1337)
    graph = Trainer(2, 3, CONFIG_HASH, seed=1337)
    graph.set_graph(True)
    losses = {"eager": [], "graph": []}
    for B, steps in ((4096, 6), (2048, 4)):
        # fixed device buffers refilled in place: the graph keys on the pointers
        pos_d = torch.empty(B, 2, device="cuda")
        tgt_d = torch.empty(B, 3, device="cuda")
        for s in range(steps):
            if B == 4096 and s == 3:
                _update_lr(eager, 5e-3)
                _update_lr(graph, 5e-3)
            pos, tgt = make_batch(B, step=s + (100 if B == 2048 else 0))
            pos_d.copy_(torch.from_numpy(pos))
            tgt_d.copy_(torch.from_numpy(tgt))
            eager.training_step(pos_d, tgt_d)
            graph.training_step(pos_d, tgt_d)
            losses["eager"].append(eager.loss())
            losses["graph"].append(graph.loss())
    torch.cuda.synchronize()
    a, b = trainer_arrays(eager), trainer_arrays(graph)
    for k in ("w32", "w16", "g16"):
        assert np.array_equal(a[k], b[k]), k
    for name, x, y in zip(("m1", "m2", "steps"), eager.optimizer_state(), graph.optimizer_state()):
        assert torch.equal(x, y), name  # the Adam moments and per-parameter step counts too
    assert losses["eager"] == losses["graph"]
    captures, replays = graph.graph_stats()
    # captures: first B (after the weight-packing first step), the learning-rate change, the new B
    assert captures >= 3 and replays >= 4, (captures, replays)
    assert graph.optimizer_step_count == eager.optimizer_step_count == 10


@pytest.mark.parametrize("engine", ["tile", "layered"])
def test_graph_replay_other_engines(torch_mod, engine):
    """The tile engine (HashGrid + W128/H4, configs[3]'s network) and the layer-wise engine (OneBlob +
    CutlassMLP) replay their whole step -- encoding pass, MLP kernel(s), reductions, grid backward,
    Adam -- as one graph, bit-identical to the eager step."""
    import copy
    torch = torch_mod
    from helpers import CONFIG_ONEBLOB
    from tinycudann import Trainer
    if engine == "tile":
        cfg = copy.deepcopy(CONFIG_HASH)
        cfg["network"].update({"n_neurons": 128, "n_hidden_layers": 4})
    else:
        cfg = copy.deepcopy(CONFIG_ONEBLOB)
        cfg["network"].update({"otype": "CutlassMLP", "n_neurons": 64, "n_hidden_layers": 2})
    eager = Trainer(2, 3, cfg, seed=1337)
    graph = Trainer(2, 3, cfg, seed=1337)
    assert eager.engine == ("fused" if engine == "tile" else "layered")
    graph.set_graph(True)
    B = 4096
    pos_d = torch.empty(B, 2, device="cuda")
    tgt_d = torch.empty(B, 3, device="cuda")
    le, lg = [], []
    for s in range(5):
        pos, tgt = make_batch(B, step=s)
        pos_d.copy_(torch.from_numpy(pos))
        tgt_d.copy_(torch.from_numpy(tgt))
        eager.training_step(pos_d, tgt_d)
        graph.training_step(pos_d, tgt_d)
        le.append(eager.loss())
        lg.append(graph.loss())
    torch.cuda.synchronize()
    a, b = trainer_arrays(eager), trainer_arrays(graph)
    for k in ("w32", "w16", "g16"):
        assert np.array_equal(a[k], b[k]), k
    assert le == lg
    captures, replays = graph.graph_stats()
    assert captures == 1 and replays == 4, (captures, replays)


def test_update_hyperparams_rejects_loss_type_change(torch_mod):
    """The loss type is fixed at construction (the reference's Loss::update_hyperparams holds no
    hyperparameters): a request to change it fails loudly instead of being ignored."""
    from tinycudann import _lib as L
    from tinycudann import Trainer
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    L.check(L.lib().tcnn_trainer_update_hyperparams(t.h, json.dumps({"loss": {"otype": "RelativeL2"}}).encode()))
    with pytest.raises(RuntimeError, match="loss type is fixed"):
        L.check(L.lib().tcnn_trainer_update_hyperparams(t.h, json.dumps({"loss": {"otype": "L2"}}).encode()))
