"""Diagnostic: print grid-forward mismatches between the HIP kernel and the oracle."""
import ctypes, json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd"), os.path.join(REPO, "tests")]
import numpy as np, torch
from helpers import CONFIG_HASH, make_batch
from oracle import oracle as O
from tinycudann import _lib as L
lib = L.lib()
enc = CONFIG_HASH["encoding"]
m = L.check_ptr(lib.tcnn_create_encoding(2, json.dumps(enc).encode(), 1))
n = lib.tcnn_module_n_params(m)
p32 = torch.zeros(n, dtype=torch.float32, device="cuda")
L.check(lib.tcnn_module_initialize_params(m, 1337, ctypes.c_void_p(p32.data_ptr()), 1.0))
for mult in (1.0, 5000.0):
    p16 = (p32 * mult).half().contiguous()
    B = 4096
    pos, _ = make_batch(B, seed=7)
    pos_d = torch.from_numpy(pos).cuda()
    out = torch.empty(B, 32, dtype=torch.float16, device="cuda")
    L.check(lib.tcnn_module_inference(m, None, B, ctypes.c_void_p(pos_d.data_ptr()), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(p16.data_ptr())))
    torch.cuda.synchronize()
    g = O.grid_cfg(enc, 2)
    ref = O.grid_fwd(g, pos, p16.cpu().numpy().view(np.uint16))
    got = out.cpu().numpy().view(np.uint16).T
    bad = np.argwhere(got != ref)
    print("mult", mult, "mismatches", len(bad))
    for (feat, i) in bad[:12]:
        l = feat // 2
        sc = np.float32(g.scales[l])
        px = [np.float32(np.float64(sc) * np.float64(pos[i, d]) + 0.5) for d in range(2)]
        print(f" level {l} f {feat%2} i {i} pos {pos[i]} scaled {px} got {np.uint16(got[feat,i]).view(np.float16)} ref {np.uint16(ref[feat,i]).view(np.float16)} res {g.res[l]} size {g.offsets[l+1]-g.offsets[l]}")
