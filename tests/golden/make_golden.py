"""Generate golden vectors from the reference model code (run in the build container only).

This script imports ``/root/reference/cgr_mpnn_3D/models/GNN.py`` *as is* (never copied) and runs
it on deterministic synthetic batches (``cgr_mpnn_3D._amd.synth``).  ``torch_geometric`` is not
installed here, so a small stand-in restating the two PyG primitives the reference calls is placed
in ``sys.modules`` first:

* ``MessagePassing.propagate(edge_index, x=None, edge_attr=h)`` -> ``message(edge_attr)`` (identity,
  ``GNN.py:143-145``) then sum-aggregation at ``edge_index[1]`` with
  ``dim_size = max(edge_index[1]) + 1`` (PyG infers the size this way when ``x`` is None);
* ``global_add_pool(x, batch)`` -> sum by graph id, ``batch=None`` -> ``x.sum(-2, keepdim=True)``.

Both use ``Tensor.scatter_add_`` exactly as PyG's ``utils.scatter(reduce='sum')`` does.

Outputs: ``tests/golden/<case>.npz`` holding inputs, the ``state_dict``, eval-mode predictions,
the train-mode (dropout p=0) ``MSELoss(sum)`` loss, every parameter gradient and the gradients
with respect to ``x`` / ``edge_attr`` (``gin_*``).  Only these data
files are committed; the reference itself never leaves this container.

    python tests/golden/make_golden.py [case ...]
"""

from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "cgr-mpnn-3d_amd"))
from cgr_mpnn_3D._amd.synth import make_batch, make_symmetric_batch  # noqa: E402

REF_GNN = "/root/reference/cgr_mpnn_3D/models/GNN.py"


# --------------------------------------------------------------------------------------------
# PyG stand-in (restated semantics, not PyG code)
# --------------------------------------------------------------------------------------------
def _scatter_sum(src: torch.Tensor, index: torch.Tensor, dim_size: int | None) -> torch.Tensor:
    if dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() > 0 else 0
    out = src.new_zeros((dim_size,) + tuple(src.shape[1:]))
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    return out.scatter_add_(0, idx, src)


def _scatter_mean(src: torch.Tensor, index: torch.Tensor, dim_size: int | None) -> torch.Tensor:
    # PyG utils.scatter(reduce="mean"): the sum divided by the count clamped to >= 1
    out = _scatter_sum(src, index, dim_size)
    cnt = torch.bincount(index, minlength=out.shape[0]).clamp(min=1).to(src.dtype)
    return out / cnt.view(-1, *([1] * (src.dim() - 1)))


class _MessagePassing(torch.nn.Module):
    def __init__(self, aggr: str = "add"):
        super().__init__()
        assert aggr in ("add", "sum", "mean"), "stand-in restates sum / mean aggregation only"
        self.aggr = aggr

    def propagate(self, edge_index, size=None, **kwargs):
        msg = self.message(kwargs["edge_attr"])
        red = _scatter_mean if self.aggr == "mean" else _scatter_sum
        return red(msg, edge_index[1], None if size is None else size[1])


def _global_add_pool(x, batch, size=None):
    if batch is None:
        return x.sum(dim=-2, keepdim=x.dim() == 2)
    return _scatter_sum(x, batch, size)


def _global_mean_pool(x, batch, size=None):
    if batch is None:
        return x.mean(dim=-2, keepdim=x.dim() == 2)
    return _scatter_mean(x, batch, size)


def _global_max_pool(x, batch, size=None):
    # PyG utils.scatter(reduce="max") without torch_scatter: scatter_reduce amax, include_self=False
    if batch is None:
        return x.max(dim=-2, keepdim=x.dim() == 2)[0]
    if size is None:
        size = int(batch.max()) + 1 if batch.numel() > 0 else 0
    idx = batch.view(-1, *([1] * (x.dim() - 1))).expand_as(x)
    return x.new_zeros((size,) + tuple(x.shape[1:])).scatter_reduce(0, idx, x, reduce="amax",
                                                                    include_self=False)


def _install_pyg_standin():
    tg = types.ModuleType("torch_geometric")
    tgnn = types.ModuleType("torch_geometric.nn")
    tgnn.MessagePassing = _MessagePassing
    tgnn.global_add_pool = _global_add_pool
    tgnn.global_mean_pool = _global_mean_pool
    tgnn.global_max_pool = _global_max_pool
    tg.nn = tgnn
    sys.modules["torch_geometric"] = tg
    sys.modules["torch_geometric.nn"] = tgnn


def load_reference_gnn():
    _install_pyg_standin()
    spec = importlib.util.spec_from_file_location("ref_cgr_gnn", REF_GNN)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class _Data:
    def __init__(self, x, edge_index, edge_attr, batch):
        self.x, self.edge_index, self.edge_attr, self.batch = x, edge_index, edge_attr, batch


ACTS = {"relu": F.relu, "silu": F.silu, "gelu": F.gelu, "tanh": torch.tanh, "sigmoid": torch.sigmoid,
        "elu": F.elu, "leaky_relu": F.leaky_relu, "softplus": F.softplus, "mish": F.mish,
        "selu": F.selu}

# name -> (batch kwargs, model kwargs, extra)
CASES = {
    # BASELINE cfg1: CGR (no MACE) depth 2, hidden 128, batch 32
    "cfg1_relu": (dict(num_graphs=32, n_atoms=30, n_bonds=30, n_mace=0, seed=11),
                  dict(depth=2, hidden=128, act="relu", skip=False), {}),
    # MACE-width input, learnable skip with non-unit sigma, SiLU
    "mace_silu_skip": (dict(num_graphs=2, n_atoms=30, n_bonds=30, n_mace=768, seed=12),
                       dict(depth=4, hidden=64, act="silu", skip=True), {}),
    # ragged atom counts, GELU(erf), depth 3
    "ragged_gelu": (dict(num_graphs=6, n_atoms=20, n_bonds=22, n_mace=16, seed=13,
                         n_atoms_jitter=12),
                    dict(depth=3, hidden=48, act="gelu", skip=False), {}),
    # one reaction, batch=None (cli_tool/activation_energy_predictor.py:72-76 call pattern)
    "single_graph_none": (dict(num_graphs=1, n_atoms=10, n_bonds=10, n_mace=0, seed=14),
                          dict(depth=2, hidden=32, act="relu", skip=False), {"batch_none": True}),
    # depth 1, H not a multiple of 16, learnable skip, ReLU
    "depth1_skip": (dict(num_graphs=5, n_atoms=12, n_bonds=14, n_mace=5, seed=15),
                    dict(depth=1, hidden=20, act="relu", skip=True), {}),
    # no edge features (GNN(num_node_features, 0), tests/test_trainer.py:37-38)
    "no_edge_features": (dict(num_graphs=3, n_atoms=9, n_bonds=10, n_mace=0, seed=16),
                         dict(depth=2, hidden=24, act="relu", skip=False), {"drop_edge_attr": True}),
    # eval mode ignores dropout (p>0): predictions must equal the p=0 network
    "eval_dropout": (dict(num_graphs=4, n_atoms=30, n_bonds=30, n_mace=32, seed=17),
                     dict(depth=3, hidden=40, act="relu", skip=False), {"eval_dropout": 0.3}),
    # denser, larger graphs (stress-shaped, small): 60 atoms / 120 bonds
    "dense_relu_skip": (dict(num_graphs=3, n_atoms=60, n_bonds=120, n_mace=64, seed=18),
                        dict(depth=4, hidden=80, act="relu", skip=True), {}),
    # DMPNNConv(aggr="mean") (GNN.py:22,63,119), ragged graphs
    "mean_aggr_relu": (dict(num_graphs=5, n_atoms=18, n_bonds=20, n_mace=16, seed=20,
                            n_atoms_jitter=6),
                       dict(depth=3, hidden=40, act="relu", skip=False), {"aggr": "mean"}),
    # pooling_fn=global_mean_pool (GNN.py:23,110), learnable skip
    "mean_pool_silu_skip": (dict(num_graphs=4, n_atoms=14, n_bonds=15, n_mace=8, seed=21,
                                 n_atoms_jitter=5),
                            dict(depth=2, hidden=36, act="silu", skip=True), {"pool": "mean"}),
    # both, one reaction with batch=None (global_mean_pool(h, None) = mean over all nodes)
    "mean_both_gelu_none": (dict(num_graphs=1, n_atoms=16, n_bonds=17, n_mace=0, seed=22),
                            dict(depth=2, hidden=24, act="gelu", skip=False),
                            {"aggr": "mean", "pool": "mean", "batch_none": True}),
    # pooling_fn=global_max_pool, smooth activation (no ties), ragged graphs
    "max_pool_silu": (dict(num_graphs=5, n_atoms=16, n_bonds=18, n_mace=8, seed=23,
                           n_atoms_jitter=6),
                      dict(depth=3, hidden=32, act="silu", skip=False), {"pool": "max"}),
    # global_max_pool over symmetric atoms (identical leaves on one atom): columns a leaf wins are
    # ties, whose gradient scatter_reduce("amax") shares evenly
    "max_pool_ties_silu": (dict(num_graphs=4, n_leaves=3, n_chain=6, n_mace=8, seed=24,
                                symmetric=True),
                           dict(depth=2, hidden=32, act="silu", skip=False), {"pool": "max"}),
    # the same with batch=None: x.max(dim=-2), whose gradient goes to the first arg-max only
    "max_pool_ties_none": (dict(num_graphs=1, n_leaves=3, n_chain=5, n_mace=8, seed=25,
                                symmetric=True),
                           dict(depth=2, hidden=24, act="gelu", skip=False),
                           {"pool": "max", "batch_none": True}),
}
# activation_fn beyond train.py's three (the reference applies any callable, GNN.py:86,127): one
# small ragged case per further activation, alternating skip / aggregation / pooling
for _i, (_act, _skip, _ex) in enumerate([("tanh", True, {}), ("sigmoid", False, {"aggr": "mean"}),
                                         ("elu", True, {}), ("leaky_relu", False, {}),
                                         ("softplus", True, {"pool": "mean"}),
                                         ("mish", False, {}), ("selu", True, {})]):
    CASES[f"act_{_act}"] = (dict(num_graphs=3, n_atoms=12, n_bonds=13, n_mace=8, seed=40 + _i,
                                 n_atoms_jitter=4),
                            dict(depth=2, hidden=24, act=_act, skip=_skip), _ex)


def run_case(ref, name, bkw, mkw, extra):
    if bkw.get("symmetric"):
        b = make_symmetric_batch(**{k: v for k, v in bkw.items() if k != "symmetric"})
    else:
        b = make_batch(**bkw)
    x = torch.from_numpy(b.x)
    ei = torch.from_numpy(b.edge_index)
    ea = torch.from_numpy(b.edge_attr)
    if extra.get("drop_edge_attr"):
        ea = ea[:, :0].contiguous()
    batch = None if extra.get("batch_none") else torch.from_numpy(b.batch)
    y = torch.from_numpy(b.y)
    D, H = mkw["depth"], mkw["hidden"]

    torch.manual_seed(1000 + len(name))
    p_eval = extra.get("eval_dropout", 0.0)
    kw = {}
    if extra.get("aggr"):
        kw["aggr"] = extra["aggr"]
    if extra.get("pool") == "mean":
        kw["pooling_fn"] = _global_mean_pool
    if extra.get("pool") == "max":
        kw["pooling_fn"] = _global_max_pool
    model = ref.GNN(x.shape[1], ea.shape[1], depth=D, hidden_sizes=[H] * D,
                    dropout_ps=[p_eval] * D, activation_fn=ACTS[mkw["act"]],
                    use_learnable_skip=mkw["skip"], **kw)
    if mkw["skip"]:
        with torch.no_grad():
            for i, w in enumerate(model.skip_weights):
                w.fill_(0.6 + 0.3 * i)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}

    data = _Data(x, ei, ea, batch)
    model.eval()
    with torch.no_grad():
        y_eval = model(data)
    # train-mode fwd+bwd with dropout disabled so gradients are deterministic
    model.dropout_ps = [0.0] * D
    model.train()
    model.zero_grad()
    # inputs that require grad: autograd's x.grad / edge_attr.grad (through x[row] and
    # cat([x, s]), GNN.py:85-86,105-106) become the gin_* vectors
    xg = x.clone().requires_grad_(True)
    eag = ea.clone().requires_grad_(True)
    pred = model(_Data(xg, ei, eag, batch))
    loss = torch.nn.MSELoss(reduction="sum")(pred, y.view_as(pred))
    loss.backward()

    out = {
        "in_x": b.x, "in_edge_index": b.edge_index, "in_edge_attr": ea.numpy(),
        "in_batch": b.batch, "in_ptr": b.ptr, "in_y": b.y,
        "out_y_eval": y_eval.numpy(), "out_y_train": pred.detach().numpy(),
        "out_loss": np.asarray(loss.item(), dtype=np.float64),
    }
    for k, v in sd.items():
        out["p_" + k] = v.numpy()
    for k, p in model.named_parameters():
        out["g_" + k] = p.grad.numpy()
    out["gin_x"] = xg.grad.numpy()
    out["gin_edge_attr"] = (eag.grad if eag.grad is not None else torch.zeros_like(ea)).numpy()
    meta = dict(name=name, depth=D, hidden=H, act=mkw["act"], skip=mkw["skip"],
                aggr=extra.get("aggr", "add"), pool=extra.get("pool", "add"),
                batch_none=bool(extra.get("batch_none")), eval_dropout=p_eval,
                num_node_features=int(x.shape[1]), num_edge_features=int(ea.shape[1]),
                generator="cgr_mpnn_3D._amd.synth.make_batch", batch_kwargs=bkw,
                reference="cgr_mpnn_3D/models/GNN.py (tobjec/CGR-MPNN-3D @ 2025-02-27)",
                torch=torch.__version__)
    out["meta"] = np.asarray(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(f"{name}: N={x.shape[0]} E={ei.shape[1]} y_eval[:3]={y_eval[:3].tolist()} "
          f"loss={loss.item():.6g}")


def isolated_last_node_case(ref):
    """Record the reference's failure when the batch's last node has no incoming edge."""
    b = make_batch(num_graphs=2, n_atoms=8, n_bonds=8, n_mace=0, seed=19)
    # append one isolated atom to the last graph
    x = np.concatenate([b.x, b.x[-1:]], 0)
    batch = np.concatenate([b.batch, b.batch[-1:]], 0)
    ptr = b.ptr.copy()
    ptr[-1] += 1
    torch.manual_seed(7)
    model = ref.GNN(x.shape[1], b.edge_attr.shape[1], depth=2, hidden_sizes=[16, 16],
                    dropout_ps=[0.0, 0.0])
    model.eval()
    err = ""
    try:
        with torch.no_grad():
            model(_Data(torch.from_numpy(x), torch.from_numpy(b.edge_index),
                        torch.from_numpy(b.edge_attr), torch.from_numpy(batch)))
    except Exception as e:  # noqa: BLE001 - we record what the reference raises
        err = type(e).__name__
    np.savez_compressed(os.path.join(HERE, "isolated_last_node.npz"), in_x=x,
                        in_edge_index=b.edge_index, in_edge_attr=b.edge_attr, in_batch=batch,
                        in_ptr=ptr, ref_error=np.asarray(err))
    print("isolated_last_node: reference raised", err)


def main(names=None):
    """names: the cases to (re)generate (default: all, plus isolated_last_node)."""
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ref = load_reference_gnn()
    for name, (bkw, mkw, extra) in CASES.items():
        if not names or name in names:
            run_case(ref, name, bkw, mkw, extra)
    if not names or "isolated_last_node" in names:
        isolated_last_node_case(ref)


if __name__ == "__main__":
    main(sys.argv[1:])
