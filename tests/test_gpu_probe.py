"""MFMA f32_16x16x32_f16 operand/accumulator maps and ds_read_b64_tr_b16 semantics, checked with
exact integer data on the device (the fused MLP kernel's fragment layout rests on these)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_mfma_and_transpose_read_layout():
    import torch
    from tinycudann import _lib as L
    mf = torch.zeros(64 * 4, dtype=torch.float32, device="cuda")
    tr = torch.zeros(64 * 8, dtype=torch.int16, device="cuda")
    L.check(L.lib().tcnn_debug_probe(None, ctypes.c_void_p(mf.data_ptr()), ctypes.c_void_p(tr.data_ptr())))
    torch.cuda.synchronize()
    mf = mf.cpu().numpy().reshape(64, 4)
    tr = tr.cpu().numpy().reshape(64, 8)
    A = np.array([[((i * 3 + k * 5) % 11) - 5 for k in range(32)] for i in range(16)], dtype=np.float64)
    Bm = np.array([[((k * 7 + j * 2) % 13) - 6 for j in range(16)] for k in range(32)], dtype=np.float64)
    C = A @ Bm
    for l in range(64):
        for r in range(4):
            assert mf[l, r] == C[4 * (l >> 4) + r, l & 15], (l, r)
        for e in range(8):
            assert tr[l, e] == (8 * (l >> 4) + e) * 64 + (l & 15), (l, e)
