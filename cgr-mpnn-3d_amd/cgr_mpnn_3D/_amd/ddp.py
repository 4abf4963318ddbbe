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
        self.captured = 0  # bucket collectives recorded into a stream capture (teardown checks)

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
        """Drop the communication streams and bucket events (teardown, before
        ``dist.destroy_process_group``: see ``teardown``).  The caller has synchronised the
        device; no event is queried or synchronised here -- after a capture the events' last
        records live in a graph, and a host wait on them is not meaningful."""
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
        if torch.cuda.is_current_stream_capturing():
            self.captured += len(buckets)
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


def teardown(model=None, graphs_released: bool = False):
    """End data parallelism in a fixed order that depends on no garbage collection, then destroy
    the process group.

    Order: (1) the caller drops every captured graph that recorded a collective (and any bound
    ``g.replay``) BEFORE calling this -- a captured collective leaves RCCL state tied to its graph
    (a graph user object, ``hipGraphRetainUserObject``, that hands the captured launch plan back
    to the communicator when the graph is destroyed), so those graphs must die while the
    communicator lives (round 3 destroyed the communicator first and aborted at interpreter
    exit); (2) the device is synchronised; (3) the gradient hook's streams and events are dropped
    (``GradAllReduce.close``) and the device synchronised again; (4) the ranks meet at a barrier;
    (5) the process group is destroyed; (6) only then is garbage collected.

    No collection runs while the communicator is alive (round 4 collected here, between (2) and
    (3)).  A captured step leaves no graph, event or tensor in a reference cycle
    (``tools/rccl_teardown_probe.py``: the collector finds only ctypes type objects after it), so
    a collection at that point freed nothing of this process group's and only re-ordered the
    release of EARLIER work's objects against the communicator's own threads -- which is where
    the one round-4 abort struck (on a native thread, not in a destructor the
    collector ran).  ``cgr_debug_abort_backtrace`` prints the native stack of any such abort.

    ``graphs_released``: the caller's statement that step (1) is done.  When the model's hook
    recorded collectives into a capture and the caller does not say so, a RuntimeWarning names
    the precondition before the communicator is destroyed (no live graph can be enumerated from
    here: torch keeps no registry of CUDAGraph objects)."""
    import gc

    if not dist.is_initialized():
        return
    hook = getattr(model, "_grad_bucket_hook", None) if model is not None else None
    if getattr(hook, "captured", 0) and not graphs_released:
        import warnings

        warnings.warn(
            "ddp.teardown: the gradient hook recorded RCCL collectives into a captured graph; "
            "drop every such graph (and any bound g.replay) before teardown and pass "
            "graphs_released=True -- a captured collective's graph destroyed after the "
            "communicator releases its RCCL state against a freed communicator", RuntimeWarning,
            stacklevel=2)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if model is not None:
        remove_grad_allreduce(model)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if dist.get_world_size() > 1:
        dist.barrier()
    dist.destroy_process_group()
    gc.collect()


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
