"""ORACLE (test infrastructure only) - torch-CPU restatement of the reference op sequence.

This is the CPU baseline ``bench.py`` times (``cpu_baseline.kind = "port"``): the same ATen op
sequence ``cgr_mpnn_3D/models/GNN.py:76-145`` executes on the reference's CPU path, with PyG's two
sum-scatters (``MessagePassing.propagate`` at ``GNN.py:134`` and ``global_add_pool`` at
``GNN.py:110``) restated as ``Tensor.scatter_add_`` the way PyG's ``utils.scatter`` does it, and
autograd providing the backward exactly as it does for the reference.  It keeps the reference's
dead readout GEMM (``GNN.py:105`` discards ``lin(...)``) so the timed work is the reference's work.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may import it.
Pinned by ``tests/test_oracle_golden.py`` against the golden vectors of the reference itself.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F


def _scatter_sum(src: torch.Tensor, index: torch.Tensor, dim_size: int) -> torch.Tensor:
    out = src.new_zeros((dim_size,) + tuple(src.shape[1:]))
    return out.scatter_add_(0, index.view(-1, 1).expand_as(src), src)


class TorchRestatement(torch.nn.Module):
    """Parameters named exactly like the reference ``state_dict``."""

    def __init__(self, state_dict: dict, depth: int, act=F.relu, learnable_skip=False,
                 dropout_ps=None, keep_dead_gemm: bool = True):
        super().__init__()
        self.depth = depth
        self.act = act
        self.learnable_skip = learnable_skip
        self.dropout_ps = dropout_ps or [0.0] * depth
        self.keep_dead_gemm = keep_dead_gemm
        self.params = torch.nn.ParameterDict(
            {k.replace(".", "__"): torch.nn.Parameter(torch.as_tensor(v).clone().float())
             for k, v in state_dict.items()})

    def p(self, key):
        return self.params[key.replace(".", "__")]

    def forward(self, x, edge_index, edge_attr, batch, num_graphs=None):
        row, col = edge_index[0], edge_index[1]
        n_prime = int(col.max()) + 1  # PyG's inferred dim_size (x=None at GNN.py:134)
        h0 = self.act(F.linear(torch.cat([x[row], edge_attr], 1), self.p("edge_init.weight"),
                               self.p("edge_init.bias")))
        h = h0
        for l in range(self.depth):
            a = _scatter_sum(h, col, n_prime)
            rev = torch.flip(h.view(h.size(0) // 2, 2, -1), dims=[1]).view(h.size(0), -1)
            h = F.linear(a[row] - rev, self.p(f"convs.{l}.lin.weight"),
                         self.p(f"convs.{l}.lin.bias"))
            if self.learnable_skip:
                h = h + self.p(f"skip_weights.{l}") * h0
            else:
                h = h + h0
            h = F.dropout(self.act(h), self.dropout_ps[l], training=self.training)
        l = self.depth - 1
        s = _scatter_sum(h, col, n_prime)
        if self.keep_dead_gemm:  # the reference computes and discards this (GNN.py:105,141)
            rev = torch.flip(h.view(h.size(0) // 2, 2, -1), dims=[1]).view(h.size(0), -1)
            _ = F.linear(s[row] - rev, self.p(f"convs.{l}.lin.weight"),
                         self.p(f"convs.{l}.lin.bias"))
        hn = self.act(F.linear(torch.cat([x, s], 1), self.p("edge_to_node.weight"),
                               self.p("edge_to_node.bias")))
        if batch is None:
            g = hn.sum(dim=-2, keepdim=True)
        else:
            B = num_graphs if num_graphs is not None else int(batch.max()) + 1
            g = _scatter_sum(hn, batch, B)
        return F.linear(g, self.p("ffn.weight"), self.p("ffn.bias")).squeeze(-1)


def random_state_dict(num_node_features: int, num_edge_features: int, hidden: int, depth: int,
                      learnable_skip: bool = False, seed: int = 0) -> dict:
    """Reference-shaped parameters with nn.Linear's default init (GNN.py:53-74)."""
    g = torch.Generator().manual_seed(seed)

    def lin(i, o):
        bound = 1.0 / (i ** 0.5)
        w = (torch.rand(o, i, generator=g) * 2 - 1) * bound
        b = (torch.rand(o, generator=g) * 2 - 1) * bound
        return w, b

    sd = {}
    sd["edge_init.weight"], sd["edge_init.bias"] = lin(num_node_features + num_edge_features,
                                                       hidden)
    for l in range(depth):
        sd[f"convs.{l}.lin.weight"], sd[f"convs.{l}.lin.bias"] = lin(hidden, hidden)
    sd["edge_to_node.weight"], sd["edge_to_node.bias"] = lin(num_node_features + hidden, hidden)
    sd["ffn.weight"], sd["ffn.bias"] = lin(hidden, 1)
    if learnable_skip:
        for l in range(depth):
            sd[f"skip_weights.{l}"] = torch.tensor(1.0)
    return sd
