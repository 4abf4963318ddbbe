"""Pooling functions accepted as ``GNN(pooling_fn=...)`` (the reference default is PyG's
``global_add_pool``, ``GNN.py:5,23,110``).  The native path fuses add-pooling with the ffn head, so
``pooling_fn`` is only inspected to select that fused head; these functions also work standalone.
"""

from __future__ import annotations

import torch


def global_add_pool(x: torch.Tensor, batch: torch.Tensor | None, size: int | None = None):
    """Sum node rows per graph id (PyG semantics: ``batch=None`` -> ``x.sum(-2, keepdim)``)."""
    if batch is None:
        return x.sum(dim=-2, keepdim=x.dim() == 2)
    if size is None:
        size = int(batch.max()) + 1 if batch.numel() else 0
    out = x.new_zeros((size,) + tuple(x.shape[1:]))
    return out.index_add_(0, batch, x)


def is_add_pool(fn) -> bool:
    """True for this module's global_add_pool or PyG's (matched by name, PyG may be absent)."""
    return fn is global_add_pool or getattr(fn, "__name__", "") == "global_add_pool"
