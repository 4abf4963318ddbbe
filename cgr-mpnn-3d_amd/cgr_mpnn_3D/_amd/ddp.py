"""Data parallelism over the GPUs of one node: graph-sharded batches + bucketed RCCL all-reduce.

The reference trains on one device (``train.py:109-114``, ``trainer.py:138-144``).  Reactions are
disconnected graphs, so a global batch shards by whole reaction graphs with no cross-rank edges
(SURVEY.md §8e); the only exchange per step is the gradient sum.  The native backward writes
every parameter gradient into one flat fp32 buffer laid out in all-reduce bucket order
(``functional.grad_layout``: edge_to_node + ffn, then the layers from the top down, then
edge_init + skip weights -- the order in which the backward finishes them) and records a ready
event per bucket.  ``GradAllReduce`` starts each bucket's ``all_reduce(SUM)`` on a communication
stream as soon as its event fires, so the collectives of the readout and the upper layers run
over RCCL/xGMI while the lower layers' backward still computes; the caller's stream then waits
for the last one before the optimizer reads the gradients.  Everything is stream-ordered (no host
wait), so the whole step, collectives included, is captured into one HIP graph.

SUM, not AVG: the reference loss is ``MSELoss(reduction="sum")`` (``train.py:120``), so summing
per-rank gradients reproduces the single-process gradient of the whole global batch.
"""

from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist


class GradAllReduce:
    """Bucket hook: ``all_reduce(SUM)`` of every gradient bucket over `group`.

    On CUDA tensors with events, bucket b's collective is enqueued on a per-device communication
    stream after waiting for its ready event (overlapping the rest of the backward), and the
    caller's stream waits for the communication stream at the end.  Without events (CPU / gloo
    tests) the buckets are reduced in order on the caller's stream.  `op` replaces the collective
    (tests: a scaling op shows which bucket ran after which event)."""

    def __init__(self, group=None, op=None):
        self.group = group
        self.op = op
        self._streams = {}
        self._events = {}

    def bucket_events(self, dev, n):
        key = (dev.index if dev.index is not None else torch.cuda.current_device(), n)
        evs = self._events.get(key)
        if evs is None:
            evs = [torch.cuda.Event() for _ in range(n)]
            with torch.cuda.device(key[0]):
                s = torch.cuda.current_stream()
                for e in evs:  # materialise the hipEvent_t handles (created on first record)
                    e.record(s)
            self._events[key] = evs
        return evs

    def _reduce(self, t):
        if self.op is not None:
            self.op(t)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def close(self):
        """Synchronise and drop the communication streams and bucket events (teardown, before
        ``dist.destroy_process_group``: see ``teardown``)."""
        for st in self._streams.values():
            st.synchronize()
        for evs in self._events.values():
            for e in evs:
                e.synchronize()
        self._streams.clear()
        self._events.clear()

    def __call__(self, flat, buckets, events):
        if events is None or not flat.is_cuda:
            for a, b in buckets:
                self._reduce(flat[a:b])
            return
        dev = flat.device
        cur = torch.cuda.current_stream(dev)
        cs = self._streams.get(dev)
        if cs is None:
            cs = self._streams[dev] = torch.cuda.Stream(dev)
        for (a, b), ev in zip(buckets, events):
            cs.wait_event(ev)
            with torch.cuda.stream(cs):
                self._reduce(flat[a:b])
        cur.wait_stream(cs)


def install_grad_allreduce(model, group=None, op=None):
    """Sum the model's gradient buckets across `group` inside every native backward."""
    model._grad_bucket_hook = GradAllReduce(group, op)
    return model


def remove_grad_allreduce(model):
    hook = getattr(model, "_grad_bucket_hook", None)
    if hook is not None and hasattr(hook, "close"):
        hook.close()
    model._grad_bucket_hook = None
    return model


def _collect_verbosely():
    """Diagnostic (CGR_TEARDOWN_DIAG=1): free the collector's garbage one object at a time,
    naming each on stderr first, so an abort inside the collection names its object."""
    import gc
    import sys

    gc.set_debug(gc.DEBUG_SAVEALL)
    gc.collect()
    gc.set_debug(0)
    junk = list(gc.garbage)
    gc.garbage.clear()
    print(f"[teardown] {len(junk)} collectable objects", file=sys.stderr, flush=True)
    while junk:
        o = junk.pop()
        t = type(o)
        if "torch" in t.__module__ or "cgr" in t.__module__ or t.__name__ in ("Event", "Stream"):
            print(f"[teardown] freeing {t.__module__}.{t.__qualname__}", file=sys.stderr,
                  flush=True)
        del o
        gc.collect()
    print("[teardown] garbage freed", file=sys.stderr, flush=True)


def teardown(model=None):
    """End data parallelism in the order the communicator needs, then destroy the process group.

    A collective captured into a HIP graph leaves RCCL state tied to that graph: RCCL attaches a
    destructor (a graph user object, ``hipGraphRetainUserObject``) that hands the captured
    collective's launch plan back to its communicator when the graph is destroyed.  Destroying
    the communicator while such a graph is alive -- what ``bench.py`` did (round 3: the captured
    step ``g`` was still referenced at ``destroy_process_group``) -- lets that destructor run
    against a freed communicator later, at interpreter exit: an intermittent abort after all the
    work had succeeded.  So, in this order: the caller drops every captured graph that recorded a
    collective (and any bound ``g.replay``) BEFORE calling this; here the device is synchronised,
    reference cycles are collected (the graph destructors run now, while the communicator lives),
    the device is synchronised again, the gradient hook's communication streams and events are
    released, the ranks meet at a barrier and only then is the process group destroyed."""
    import gc

    if not dist.is_initialized():
        return
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if os.environ.get("CGR_TEARDOWN_DIAG") == "1":
        _collect_verbosely()
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if model is not None:
        remove_grad_allreduce(model)
    if dist.get_world_size() > 1:
        dist.barrier()
    dist.destroy_process_group()


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
