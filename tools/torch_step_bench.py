"""Throughput of the torch training step (the NeuralBTF caller's path) beside the Trainer path, on
config_hash.json at B = 2^16 and 2^18 (the reference documents its binding
overhead, README.md:130-132, "~2x slower" at 64k).

torch step = the reference's samples/mlp_learning_an_image_pytorch.py:159-170 loop body:
tinycudann.NetworkWithInputEncoding forward (Module forward that keeps its encoding), the relative L2
written in torch, loss.backward() (Module backward on the kept encoding), torch.optim.Adam.step() on
the fp32 parameters. Trainer step = one tcnn_trainer_training_step (fused kernel, grid backward +
network Adam, grid Adam). Synthetic uniform positions and analytic targets resident in HBM;
torch.cuda events around K steps after W warm-up steps. Also reports the torch step with the forward
context disabled (backward recomputes the forward: TCNN_NO_FORWARD_KEEP=1) for the A/B, in the same
process (the switch is read when a module is built, so the A/B builds a second model under it).

  python tools/torch_step_bench.py [--out profiles/r03_torch_step.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]


def run(iters, graph):
    import torch
    from bench import rgb_field_torch
    import tinycudann as tcnn
    from tinycudann import Trainer

    def timed(fn, iters, warm=10):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / iters * 1e-3

    cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
    rows = []
    for lb in (16, 18, 20):
        B = 1 << lb
        pos = torch.rand(B, 2, device="cuda")
        tgt = rgb_field_torch(pos)
        model = tcnn.NetworkWithInputEncoding(2, 3, cfg["encoding"], cfg["network"]).cuda()
        opt = torch.optim.Adam(model.parameters(), lr=0.01)

        def make_step(model, opt):
            def torch_step():
                out = model(pos)
                loss = ((out - tgt.to(out.dtype)) ** 2 / (out.detach() ** 2 + 0.01)).mean()
                opt.zero_grad()
                loss.backward()
                opt.step()
            return torch_step

        os.environ["TCNN_NO_FORWARD_KEEP"] = "1"  # read when the module is built: the backward recomputes the forward
        model_rc = tcnn.NetworkWithInputEncoding(2, 3, cfg["encoding"], cfg["network"]).cuda()
        os.environ.pop("TCNN_NO_FORWARD_KEEP", None)
        opt_rc = torch.optim.Adam(model_rc.parameters(), lr=0.01)
        s_torch = timed(make_step(model, opt), iters)
        s_recompute = timed(make_step(model_rc, opt_rc), iters)
        s_keep2 = timed(make_step(model, opt), iters)  # again, to see the drift between the two measurements
        t = Trainer(2, 3, cfg, seed=1337)
        if graph:
            t.set_graph(True)
        s_tr = timed(lambda: t.training_step(pos, tgt), iters)
        rows.append({"batch": B, "torch_step_s": s_torch, "torch_steps_per_s": 1 / s_torch, "trainer_step_s": s_tr,
                     "trainer_steps_per_s": 1 / s_tr, "torch_over_trainer": s_torch / s_tr,
                     "torch_step_recompute_s": s_recompute, "torch_step_keep_again_s": s_keep2,
                     "module_engine": model.native_tcnn_module.engine(),
                     "module_inference_engine": model.native_tcnn_module.inference_engine()})
        print(json.dumps(rows[-1]), flush=True)
        del model, opt, t, model_rc, opt_rc
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        run(args.iters, args.graph)
        return
    res = {"what": "torch NetworkWithInputEncoding training step (reference samples/mlp_learning_an_image_pytorch.py:159-170) "
                   "vs Trainer::training_step, config_hash.json; torch_step: Module forward keeps its encoding for the "
                   "backward; torch_step_recompute: TCNN_NO_FORWARD_KEEP=1 (backward recomputes the forward)",
           "rows": run(args.iters, args.graph)}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
