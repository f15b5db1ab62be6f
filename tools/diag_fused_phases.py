"""Diagnostic: wave-cycle split of the fused kernel's slice loop (s_memtime stamps build)."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd"), os.path.join(REPO, "tests")]
import torch
from helpers import CONFIG_HASH
from tinycudann import Trainer, _lib as L
B = 1 << int(os.environ.get("LOG2B", "18"))
t = Trainer(2, 3, CONFIG_HASH)
pos = torch.rand(B, 2, device="cuda"); tgt = torch.rand(B, 3, device="cuda")
out = (ctypes.c_uint64 * 16)()
for _ in range(3):
    L.check(L.lib().tcnn_debug_fused_phase_cycles(t.h, None, B, ctypes.c_void_p(pos.data_ptr()), ctypes.c_void_p(tgt.data_ptr()), out))
tot = sum(out)
nw = min(B // 128, 512) * 4  # workgroups (fused_train_n_blocks) x 4 waves
names = ["grid encode (gathers)", "hidden fwd", "out layer + loss", "bwd hidden + dW", "dW0 (first layer)", "dL/dx + store",
         "prologue (per wave)", "epilogue reduce (per wave)", "barrier wait (per wave)",
         "  reduce: waves 2,3 write", "  reduce: waves 0,1 add + write", "  reduce: final add + slab store"]
for n, v in zip(names, out):
    print(f"{n:28s} {v/tot*100:5.1f}%  {v/ (B/32):8.0f} cycles/slice  {v/nw:8.0f} cycles/wave  {v/nw/2400:8.2f} us/wave@2.4GHz")
