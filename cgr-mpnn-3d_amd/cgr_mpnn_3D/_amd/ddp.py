"""Data parallelism over the GPUs of one node: graph-sharded batches + one RCCL all-reduce.

The reference trains on one device (``train.py:109``).  Reactions are disconnected graphs, so a
global batch shards by whole reaction graphs with no cross-rank edges; the only
exchange per step is the gradient sum.  The native backward writes every parameter gradient into
ONE flat fp32 bucket (``functional.GNNFunction.backward``), so the exchange is a single
``all_reduce(SUM)`` of 5.9 MB (cfg2) over RCCL/xGMI, issued on the backward's stream before
autograd hands the per-parameter views to the optimizer.

SUM, not AVG: the reference loss is ``MSELoss(reduction="sum")`` (``train.py:120``), so summing
per-rank gradients reproduces the single-process gradient of the whole global batch.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def install_grad_allreduce(model, group=None):
    """Sum the model's flat gradient bucket across `group` inside every native backward."""

    def hook(flat: torch.Tensor):
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)

    model._grad_bucket_hook = hook
    return model


def remove_grad_allreduce(model):
    model._grad_bucket_hook = None
    return model


def shard_ranges(graph_edges: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Split graphs [0, B) into `world` contiguous ranges with ~equal edge counts.

    Greedy on the prefix sum: rank r takes graphs up to the first prefix >= (r+1)/world of the
    total.  Every rank gets >= 1 graph when B >= world.
    """
    B = int(graph_edges.shape[0])
    if world <= 0:
        raise ValueError("world must be >= 1")
    if B < world:
        raise ValueError(f"cannot shard {B} graphs over {world} ranks")
    csum = np.cumsum(graph_edges, dtype=np.float64)
    total = csum[-1] if B else 0.0
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        k = int(np.searchsorted(csum, target, side="left")) + 1
        k = max(k, bounds[-1] + 1)  # at least one graph per rank
        k = min(k, B - (world - r))  # leave one graph for every remaining rank
        bounds.append(k)
    bounds.append(B)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def shard_batch(batch, rank: int, world: int):
    """The `rank`-th shard of a collated RxnBatch (numpy, PyG layout), re-based to start at 0."""
    from .synth import RxnBatch

    src = batch.edge_index[0]
    gid_of_edge = batch.batch[src]
    graph_edges = np.bincount(gid_of_edge, minlength=batch.num_graphs)
    g0, g1 = shard_ranges(graph_edges, world)[rank]
    v0, v1 = int(batch.ptr[g0]), int(batch.ptr[g1])
    emask = (gid_of_edge >= g0) & (gid_of_edge < g1)
    return RxnBatch(x=batch.x[v0:v1].copy(), edge_index=(batch.edge_index[:, emask] - v0).copy(),
                    edge_attr=batch.edge_attr[emask].copy(), batch=batch.batch[v0:v1] - g0,
                    ptr=batch.ptr[g0:g1 + 1] - v0, y=batch.y[g0:g1].copy())
