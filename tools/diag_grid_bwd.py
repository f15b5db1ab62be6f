"""Diagnostic: grid backward through the C-ABI (grid-only Module, AoS dL/dy) vs the oracle, per level,
at several dL/dy magnitudes; then the NetworkWithInputEncoding module backward per level."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd"), os.path.join(REPO, "tests")]
from helpers import CONFIG_HASH, make_batch, rel_err  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tinycudann import _lib as L  # noqa: E402

lib = L.lib()
enc = CONFIG_HASH["encoding"]
g = O.grid_cfg(enc, 2)
m = L.check_ptr(lib.tcnn_create_encoding(2, json.dumps(enc).encode(), 1))
n = lib.tcnn_module_n_params(m)
W = lib.tcnn_module_n_output_dims(m)
p16 = torch.zeros(n, dtype=torch.float16, device="cuda")
sizes = [256, 576, 1296, 2920, 6568, 14888] + [32768] * 10
offs = np.concatenate([[0], np.cumsum(sizes)]) * 2
for B in (65536,):
    for mag in (1e-4, 1e-2, 1.0):
        pos, _ = make_batch(B, seed=11)
        rng = np.random.default_rng(1)
        dy = (rng.standard_normal((B, W)) * mag).astype(np.float16)
        pos_d = torch.from_numpy(pos).cuda()
        dy_d = torch.from_numpy(dy).cuda()
        grad = torch.empty(n, dtype=torch.float16, device="cuda")
        out = torch.empty(B, W, dtype=torch.float16, device="cuda")
        ctx = L.check_ptr(lib.tcnn_module_forward(m, None, B, ctypes.c_void_p(pos_d.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                                  ctypes.c_void_p(p16.data_ptr()), 0))
        L.check(lib.tcnn_module_backward(m, None, ctx, B, None, ctypes.c_void_p(dy_d.data_ptr()), ctypes.c_void_p(grad.data_ptr()),
                                         ctypes.c_void_p(pos_d.data_ptr()), None, ctypes.c_void_p(p16.data_ptr())))
        torch.cuda.synchronize()
        soa = np.ascontiguousarray(dy.T[:32]).view(np.uint16)
        ref = O.grid_bwd(g, pos, soa)
        got = grad.float().cpu().numpy()
        per = [rel_err(got[offs[l]:offs[l + 1]], ref[offs[l]:offs[l + 1]]) for l in range(16)]
        print(f"B={B} mag={mag}: total {rel_err(got, ref):.2e}  per-level " + " ".join(f"{e:.1e}" for e in per))

# NetworkWithInputEncoding module backward (fused kernel with external dL/doutput)
net = CONFIG_HASH["network"]
mm = L.check_ptr(lib.tcnn_create_network_with_input_encoding(2, 3, json.dumps(enc).encode(), json.dumps(net).encode()))
n = lib.tcnn_module_n_params(mm)
p32 = torch.zeros(n, dtype=torch.float32, device="cuda")
L.check(lib.tcnn_module_initialize_params(mm, 42, ctypes.c_void_p(p32.data_ptr()), 1.0))
p16 = p32.half().contiguous()
nm = O.mlp_n_params(64, 32, 2, 16)
for B in (1024, 4096, 65536):
    for mag in (0.05, 5.0):
        pos, _ = make_batch(B, seed=11)
        pos_d = torch.from_numpy(pos).cuda()
        out = torch.empty(B, 16, dtype=torch.float16, device="cuda")
        ctx = L.check_ptr(lib.tcnn_module_forward(mm, None, B, ctypes.c_void_p(pos_d.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                                  ctypes.c_void_p(p16.data_ptr()), 0))
        rng = np.random.default_rng(0)
        dout = np.zeros((B, 16), np.float32)
        dout[:, :3] = rng.standard_normal((B, 3)) * mag
        dout16 = torch.from_numpy(dout).half().cuda()
        grad = torch.empty(n, dtype=torch.float16, device="cuda")
        L.check(lib.tcnn_module_backward(mm, None, ctx, B, None, ctypes.c_void_p(dout16.data_ptr()), ctypes.c_void_p(grad.data_ptr()),
                                         ctypes.c_void_p(pos_d.data_ptr()), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(p16.data_ptr())))
        torch.cuda.synchronize()
        params16 = p16.cpu().numpy().view(np.uint16)
        encv = O.grid_fwd(g, pos, params16[nm:])
        outr, hidden = O.mlp_fwd(64, 32, 2, 16, params16[:nm], encv)
        wg, denc = O.mlp_bwd(64, 32, 2, 16, params16[:nm], encv, hidden, dout16.cpu().numpy().view(np.uint16))
        gg = O.grid_bwd(g, pos, denc)
        got = grad.float().cpu().numpy()
        per = [rel_err(got[nm + offs[l]:nm + offs[l + 1]], gg[offs[l]:offs[l + 1]]) for l in range(16)]
        print(f"NWIE B={B} mag={mag}: mlp {rel_err(got[:nm], wg):.2e} grid {rel_err(got[nm:], gg):.2e} per-level " + " ".join(f"{e:.1e}" for e in per))
        print("   max|denc| oracle", float(np.max(np.abs(O.h2f(denc)))), " grad absmax", float(np.max(np.abs(gg))))
        lib.tcnn_context_destroy(ctx)
