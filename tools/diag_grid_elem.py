"""Diagnostic: per-element grid-gradient mismatches of the Module backward vs the oracle -- lists
the contributing (point, corner) updates of every entry outside the bound (numpy restatement of
pos_fract / corner weights / coherent-prime hash for D = 2)."""
import sys, os, json
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "tests"),
                os.path.join(os.path.dirname(__file__), "..", "neuralbtf-tiny-cuda-nn_amd")]
import numpy as np
import torch
import test_gpu_grid_large as T
from oracle import oracle as O

enc = T.ENC_T19 if (len(sys.argv) < 2 or sys.argv[1] == "t19") else T.CONFIG_HASH["encoding"]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
got, ref, tol, g = T._module_case(torch, enc, 2, B)
L, F = g.n_levels, g.n_features_per_level
r = O.pcg32(5)
pos = O.generate_uniform(r, 2 * B).reshape(B, 2)
dy = O.h2f(T._random_dy(B, L, F, 5)).reshape(B, L, F)
tt = tol + 2.0 ** -11 * (np.abs(ref) + tol) + 2.0 ** -25
bad = np.flatnonzero(np.abs(got - ref) > tt)
print("bad", bad.size)
offs = [g.offsets[l] for l in range(L + 1)]
for p in bad[:8]:
    e = p // F
    l = int(np.searchsorted(offs, e, side="right") - 1)
    ent = e - offs[l]
    s = np.float32(g.scales[l]); res = g.res[l]; size = offs[l + 1] - offs[l]
    x = (pos.astype(np.float64) * float(s) + 0.5)
    pf = x.astype(np.float32)
    fl = np.floor(pf)
    fr = (pf - fl).astype(np.float32)
    gi = fl.astype(np.int64).astype(np.uint32)
    print(f"p={p} level={l} entry={ent} size={size} res={res} got={got[p]:.8f} ref={ref[p]:.8f} tol={tt[p]:.3e}")
    for c in range(4):
        cx = gi[:, 0] + (c & 1); cy = gi[:, 1] + ((c >> 1) & 1)
        wx = np.where(c & 1, fr[:, 0], np.float32(1) - fr[:, 0]).astype(np.float32)
        wy = np.where(c & 2, fr[:, 1], np.float32(1) - fr[:, 1]).astype(np.float32)
        w = (wx * wy).astype(np.float32)
        if res * res <= size:
            idx = (cx.astype(np.uint64) + cy.astype(np.uint64) * res) % size
        else:
            idx = (cx ^ (cy * np.uint32(2654435761))).astype(np.uint64) % size
        hit = np.flatnonzero(idx == ent)
        for i in hit:
            w16 = np.float16(w[i])
            print(f"   i={i} c={c} x={pos[i]} w={w[i]:.6e} w16={float(w16):.6e} sub={abs(float(w16)) < 6.1e-5} dy={dy[i, l, p % F]:.5f} v={float(w16) * dy[i, l, p % F]:.6e}")
