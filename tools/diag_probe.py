"""Diagnostic: ds_read_b64_tr_b16 lane mapping and packed fp16 FMA rounding behaviour."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]
import numpy as np, torch
from tinycudann import _lib as L
lib = L.lib()
mf = torch.zeros(256, dtype=torch.float32, device="cuda"); tr = torch.zeros(512, dtype=torch.int16, device="cuda")
L.check(lib.tcnn_debug_probe(None, ctypes.c_void_p(mf.data_ptr()), ctypes.c_void_p(tr.data_ptr())))
torch.cuda.synchronize()
tr = tr.cpu().numpy().reshape(64, 8).astype(np.int64)
print("tr rows (lane -> 8 elements as row,col):")
for l in [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 63]:
    print(l, [(int(v) // 64, int(v) % 64) for v in tr[l]])
rng = np.random.default_rng(0)
N = 1 << 20
a = (rng.uniform(0, 1, N)).astype(np.float16)
b = (rng.standard_normal(N) * 0.3).astype(np.float16)
c = (rng.standard_normal(N) * 0.3).astype(np.float16)
ta, tb, tc = [torch.from_numpy(x.view(np.int16)).cuda() for x in (a, b, c)]
out = torch.empty_like(ta)
L.check(lib.tcnn_debug_hfma(None, ctypes.c_void_p(ta.data_ptr()), ctypes.c_void_p(tb.data_ptr()), ctypes.c_void_p(tc.data_ptr()), ctypes.c_void_p(out.data_ptr()), N // 2))
torch.cuda.synchronize()
got = out.cpu().numpy().view(np.float16)
exact = (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float16)
dbl = (a.astype(np.float32) * b.astype(np.float32) + c.astype(np.float32)).astype(np.float16)
print("hfma: mismatches vs single-rounding", int(np.sum(got.view(np.uint16) != exact.view(np.uint16))),
      "vs fp32-then-fp16 double rounding", int(np.sum(got.view(np.uint16) != dbl.view(np.uint16))), "of", N)
