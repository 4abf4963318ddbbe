"""Experiment (checker-side, CPU): accuracy of bf16 and 3xbf16 split-precision GEMMs vs fp64.

Re-runs the oracle's forward/backward with every GEMM replaced by (x1) bf16 inputs, (x3)
hi/lo-split bf16 with three partial products, or (f32) fp32-rounded inputs, fp64 accumulate.
Result (profiles/r01_bf16_precision_experiment.txt): only fp32 inputs meet the 1e-4 parity bar.
Usage: python tools/experiments/bf16_split_precision_sim.py {f32|x3|x1}
"""
import os, sys, numpy as np, torch
_R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, _R); sys.path.insert(0, os.path.join(_R, 'cgr-mpnn-3d_amd'))
from oracle import dmpnn_numpy as on
from cgr_mpnn_3D._amd.synth import make_batch
from oracle.dmpnn_torch import random_state_dict

def bf16(a):
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
    return t.to(torch.bfloat16).to(torch.float32).numpy().astype(np.float64)
def split(a):
    a32 = np.asarray(a, np.float32).astype(np.float64)
    hi = bf16(a32); lo = bf16(a32 - hi)
    return hi, lo
MODE = sys.argv[1]
orig_matmul = np.ndarray.__matmul__
def mm(A, B):
    if MODE == 'x3':
        ah, al = split(A); bh, bl = split(B)
        return ah @ bh + ah @ bl + al @ bh
    if MODE == 'x1':
        return bf16(A) @ bf16(B)
    return np.asarray(A, np.float32).astype(np.float64) @ np.asarray(B, np.float32).astype(np.float64)

# monkeypatch: oracle uses '@' on ndarrays; wrap via a subclass-free approach: patch functions
src = open(os.path.join(_R, 'oracle', 'dmpnn_numpy.py')).read()
import types
mod = types.ModuleType('o2'); mod.__dict__['MM'] = mm
src = src.replace('q0 @ W0.T', 'MM(q0, W0.T)').replace('m @ Wl.T', 'MM(m, Wl.T)').replace('qn @ Wn.T', 'MM(qn, Wn.T)')
src = src.replace('dzn.T @ cache["qn"]', 'MM(dzn.T, cache["qn"])').replace('dzn @ Wn[:, F_:]', 'MM(dzn, Wn[:, F_:])')
src = src.replace('dz.T @ cache["ms"][l]', 'MM(dz.T, cache["ms"][l])').replace('dz @ Wl', 'MM(dz, Wl)').replace('dz0.T @ cache["q0"]', 'MM(dz0.T, cache["q0"])')
exec(compile(src, 'o2', 'exec'), mod.__dict__)
for (nb, H, D, nm) in [(32, 400, 4, 768), (16, 512, 6, 768), (32,128,2,0)]:
    b = make_batch(nb, seed=21, n_mace=nm)
    sd = {k: v.numpy().astype(np.float64) for k, v in random_state_dict(b.x.shape[1], 14, H, D, seed=0).items()}
    _, y0, g0 = on.loss_and_grads(sd, b.x, b.edge_index, b.edge_attr, b.batch, b.y, D)
    _, y1, g1 = mod.loss_and_grads(sd, b.x, b.edge_index, b.edge_attr, b.batch, b.y, D)
    ye = np.max(np.abs(y1-y0)/(np.abs(y0)+1e-6*np.abs(y0).max()))
    ge = max(np.abs(g1[k]-g0[k]).max()/np.abs(g0[k]).max() for k in g0)
    print(MODE, nb, H, D, f"y rel err {ye:.2e}  max grad rel err {ge:.2e}")
