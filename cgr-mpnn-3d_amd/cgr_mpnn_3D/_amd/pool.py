"""Pooling functions accepted as ``GNN(pooling_fn=...)`` (the reference default is PyG's
``global_add_pool``, ``GNN.py:5,23,110``; PyG's ``global_mean_pool`` and ``global_max_pool`` are
the others the native head implements).  The native path fuses pooling with the ffn head, so ``pooling_fn`` is only
inspected to select that fused head; these functions also work standalone.
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


def global_mean_pool(x: torch.Tensor, batch: torch.Tensor | None, size: int | None = None):
    """Mean of node rows per graph id (PyG semantics: sum / max(count, 1); ``batch=None`` ->
    ``x.mean(-2, keepdim)``)."""
    if batch is None:
        return x.mean(dim=-2, keepdim=x.dim() == 2)
    if size is None:
        size = int(batch.max()) + 1 if batch.numel() else 0
    out = global_add_pool(x, batch, size)
    cnt = torch.bincount(batch, minlength=size).clamp(min=1).to(x.dtype)
    return out / cnt.view(-1, *([1] * (x.dim() - 1)))


def global_max_pool(x: torch.Tensor, batch: torch.Tensor | None, size: int | None = None):
    """Column-wise max of node rows per graph id (PyG semantics: ``scatter_reduce("amax",
    include_self=False)``, 0 for a graph without nodes; ``batch=None`` -> ``x.max(-2, keepdim)``)."""
    if batch is None:
        return x.max(dim=-2, keepdim=x.dim() == 2)[0]
    if size is None:
        size = int(batch.max()) + 1 if batch.numel() else 0
    idx = batch.view(-1, *([1] * (x.dim() - 1))).expand_as(x)
    out = x.new_zeros((size,) + tuple(x.shape[1:]))
    return out.scatter_reduce(0, idx, x, reduce="amax", include_self=False)


def is_add_pool(fn) -> bool:
    """True for this module's global_add_pool or PyG's (matched by name, PyG may be absent)."""
    return fn is global_add_pool or getattr(fn, "__name__", "") == "global_add_pool"


def is_mean_pool(fn) -> bool:
    """True for this module's global_mean_pool or PyG's (matched by name)."""
    return fn is global_mean_pool or getattr(fn, "__name__", "") == "global_mean_pool"


def is_max_pool(fn) -> bool:
    """True for this module's global_max_pool or PyG's (matched by name)."""
    return fn is global_max_pool or getattr(fn, "__name__", "") == "global_max_pool"


def pooling_code(fn) -> int:
    """The native head's pooling (include/cgr_mpnn3d.h enum cgr_pooling) for ``pooling_fn``."""
    if is_add_pool(fn):
        return 0
    if is_mean_pool(fn):
        return 1
    if is_max_pool(fn):
        return 2
    raise NotImplementedError(
        f"cgr_mpnn_3D (MI355X): pooling_fn {getattr(fn, '__name__', fn)!r} has no native head; "
        "supported are global_add_pool (the reference default), global_mean_pool and "
        "global_max_pool")


def aggregation_code(aggr) -> int:
    """PyG MessagePassing aggr -> include/cgr_mpnn3d.h enum cgr_aggregation."""
    if aggr in ("add", "sum"):
        return 0
    if aggr == "mean":
        return 1
    raise NotImplementedError(
        f"cgr_mpnn_3D (MI355X): aggr={aggr!r}; the native D-MPNN implements 'add' (= 'sum', the "
        "reference default) and 'mean'")
