"""Experiment (checker-side, CPU): accuracy of fp16 two-piece split GEMMs vs the fp64 oracle.

Every GEMM of the oracle's forward/backward is replaced by the form the fp16 matrix cores would
compute (v_mfma_f32_*_f16: exact 11x11-bit products, fp32 accumulation):

  A' = A * 2^ea (power-of-two scale so max|A'| lies in [2^14, 2^15)), hi = fp16(A'),
  lo = fp16((A' - hi) * 2^11);   A B ~ 2^-(ea+eb) [hi_a hi_b + 2^-11 (hi_a lo_b + lo_a hi_b)]

with each term a float32 matmul (fp32 accumulation, like the MFMA).  Scale granularity:
  h2t  one scale per tensor;  h2r  one per row of A / per column of B (uniform along k);
  h2t4 per tensor, plus the lo.lo term;  b3  three bf16 pieces, six terms;  f32  plain float32 matmul (the exact-fp32 MFMA path).
Usage: python tools/experiments/fp16_split_precision_sim.py {f32|h2t|h2r|h2t4} [seed]
"""
import os, sys, types
import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, _R)
sys.path.insert(0, os.path.join(_R, "cgr-mpnn-3d_amd"))
from oracle import dmpnn_numpy as on  # noqa: E402
from oracle.dmpnn_torch import random_state_dict  # noqa: E402
from cgr_mpnn_3D._amd.synth import make_batch  # noqa: E402

MODE = sys.argv[1]
SEED = int(sys.argv[2]) if len(sys.argv) > 2 else 21


def _scale_exp(amax):
    amax = np.where(amax > 0, amax, 1.0)
    return 14 - np.floor(np.log2(amax))  # max|A'| in [2^14, 2^15)


def split(A, axis):
    """axis=None: per tensor; axis=1: per row (reduce over columns); axis=0: per column."""
    A = np.asarray(A, np.float32).astype(np.float64)
    if axis is None:
        e = _scale_exp(np.abs(A).max() if A.size else 1.0)
    else:
        e = _scale_exp(np.abs(A).max(axis=axis, keepdims=True))
    As = A * np.exp2(e)
    hi = As.astype(np.float16).astype(np.float64)
    lo = ((As - hi) * 2048.0).astype(np.float16).astype(np.float64)
    return hi.astype(np.float32), lo.astype(np.float32), e


def _bf16(a):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
    return t.to(torch.bfloat16).to(torch.float32).numpy()


def split_bf16x3(A):
    a = np.asarray(A, np.float32)
    p0 = _bf16(a); r = a - p0
    p1 = _bf16(r); r = r - p1
    return p0, p1, _bf16(r)


def mm_bwd(A, B):
    """b3f / b3t: backward GEMMs (all / only the weight-gradient TN ones) as bf16 hi/lo, 3 terms."""
    a, b = split_bf16x3(A), split_bf16x3(B)
    a1, b1 = a[1] + a[2], b[1] + b[2]
    a1, b1 = _bf16(a1), _bf16(b1)
    acc = (a1 @ b[0]) + (a[0] @ b1)
    return (acc + a[0] @ b[0]).astype(np.float64)


def mm(A, B):
    if MODE == "b3":  # three bf16 pieces, the six terms that reach 2^-16 |ab|, fp32 accumulation
        a, b = split_bf16x3(A), split_bf16x3(B)
        acc = np.zeros((a[0].shape[0], b[0].shape[1]), np.float32)
        for i, j in [(1, 1), (0, 2), (2, 0), (0, 1), (1, 0), (0, 0)]:
            acc = acc + a[i] @ b[j]
        return acc.astype(np.float64)
    if MODE == "f32":
        return (np.asarray(A, np.float32) @ np.asarray(B, np.float32)).astype(np.float64)
    per_row = MODE == "h2r"
    ah, al, ea = split(A, 1 if per_row else None)
    bh, bl, eb = split(B, 0 if per_row else None)
    main = ah @ bh
    corr = ah @ bl + al @ bh
    if MODE == "h2t4":
        corr = corr + (al @ bl) * np.float32(2.0 ** -11)
    out = (main.astype(np.float32) + corr.astype(np.float32) * np.float32(2.0 ** -11))
    return out.astype(np.float64) * np.exp2(-(ea + eb))


src = open(os.path.join(_R, "oracle", "dmpnn_numpy.py")).read()
BW = {"b3f": ["dzn @ Wn[:, F_:]", "dz @ Wl", 'dzn.T @ cache["qn"]', 'dz.T @ cache["ms"][l]',
             'dz0.T @ cache["q0"]'],
      "b3t": ['dzn.T @ cache["qn"]', 'dz.T @ cache["ms"][l]', 'dz0.T @ cache["q0"]']}.get(MODE, [])
if BW:
    MODE_FWD = "b3"
for a, b in [("q0 @ W0.T", "MM(q0, W0.T)"), ("m @ Wl.T", "MM(m, Wl.T)"),
             ("qn @ Wn.T", "MM(qn, Wn.T)"), ('dzn.T @ cache["qn"]', 'MM(dzn.T, cache["qn"])'),
             ("dzn @ Wn[:, F_:]", "MM(dzn, Wn[:, F_:])"),
             ('dz.T @ cache["ms"][l]', 'MM(dz.T, cache["ms"][l])'), ("dz @ Wl", "MM(dz, Wl)"),
             ('dz0.T @ cache["q0"]', 'MM(dz0.T, cache["q0"])')]:
    assert a in src, a
    src = src.replace(a, b.replace("MM(", "MMB(") if a in BW else b)
mod = types.ModuleType("o2")
mod.__dict__["MM"] = mm
mod.__dict__["MMB"] = mm_bwd
if BW:
    MODE = "b3"
exec(compile(src, "o2", "exec"), mod.__dict__)

worst_y = worst_g = 0.0
for (nb, H, D, nm, act, skip) in [(32, 400, 4, 768, "relu", False), (16, 512, 6, 768, "relu", True),
                                   (32, 128, 2, 0, "relu", False), (32, 400, 4, 768, "silu", True),
                                   (32, 400, 4, 768, "gelu", False), (64, 400, 4, 768, "relu", False)]:
    b = make_batch(nb, seed=SEED, n_mace=nm)
    sd = {k: v.numpy().astype(np.float64)
          for k, v in random_state_dict(b.x.shape[1], 14, H, D, seed=0).items()}
    if skip:
        for l in range(D):
            sd[f"skip_weights.{l}"] = np.asarray(0.5 + 0.25 * l)
    _, y0, g0 = on.loss_and_grads(sd, b.x, b.edge_index, b.edge_attr, b.batch, b.y, D, act, skip)
    _, y1, g1 = mod.loss_and_grads(sd, b.x, b.edge_index, b.edge_attr, b.batch, b.y, D, act, skip)
    ye = np.max(np.abs(y1 - y0) / (np.abs(y0) + 1e-6 * np.abs(y0).max()))
    yb = np.max(np.abs(y1 - y0) / (1e-4 * np.abs(y0) + 1e-6 * np.abs(y0).max()))  # test bar: <= 1
    gk = max(g0, key=lambda k: np.abs(g1[k] - g0[k]).max() / (np.abs(g0[k]).max() + 1e-30))
    ge = np.abs(g1[gk] - g0[gk]).max() / (np.abs(g0[gk]).max() + 1e-30)
    worst_y, worst_g = max(worst_y, ye), max(worst_g, ge)
    print(f"{MODE} B={nb} H={H} D={D} {act} skip={skip}: y rel err {ye:.2e} (bar ratio {yb:.2f})  "
          f"max grad rel err {ge:.2e} ({gk})", flush=True)
print(f"{MODE} seed={SEED} worst: y {worst_y:.2e} grad {worst_g:.2e}")
