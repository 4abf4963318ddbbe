"""autograd bridge: ``GNN.forward`` / backward -> ``cgr_gnn_forward`` / ``cgr_gnn_backward``.

The whole model step is ONE native call each way (≈25 kernel launches enqueued from C++), so the
host cost per training step is two ctypes calls plus a few caching-allocator allocations; every
launch goes to ``torch.cuda.current_stream()`` and nothing synchronises, so a training step can be
captured into a CUDA/HIP graph.
"""

from __future__ import annotations

import ctypes
from ctypes import c_float, c_void_p

import torch

from . import config as _config
from . import native


def make_config(num_node_features, num_edge_features, hidden, depth, act_code, learnable_skip,
                aggregation=0, pooling=0):
    return native.CgrGnnConfig(int(num_node_features), int(num_edge_features), int(hidden),
                               int(depth), int(act_code), 1 if learnable_skip else 0,
                               int(aggregation), int(pooling))


def _batch_struct(x, edge_index, edge_attr, batch, graph_ptr, num_graphs):
    return native.CgrBatch(
        native.ptr(x), native.ptr(edge_index),
        native.ptr(edge_attr) if edge_attr is not None and edge_attr.numel() else None,
        native.ptr(batch), native.ptr(graph_ptr),
        int(x.shape[0]), int(edge_index.shape[1]), int(num_graphs))


def _param_table(tensors):
    arr = (c_void_p * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = t.data_ptr()
    return arr


def _dropout_array(dropout_ps, depth):
    if dropout_ps is None:
        return None
    arr = (c_float * depth)()
    for i in range(depth):
        arr[i] = float(dropout_ps[i])
    return arr


def grad_layout(shapes, depth):
    """Flat gradient buffer in all-reduce bucket order (include/cgr_mpnn3d.h, CGR_GRAD_BUCKETS):
    bucket 0 = edge_to_node + ffn, 1 + k = convs.(depth-1-k), depth + 1 = edge_init + skip
    weights -- the order in which the native backward finishes them.  Every bucket starts on a
    16-byte boundary.  `shapes` are the parameter shapes in the C-ABI table order.  Returns
    (offset of each parameter, [(start, end) of each bucket], total floats)."""
    D = depth
    members = [[2 + 2 * D, 3 + 2 * D, 4 + 2 * D, 5 + 2 * D]]
    members += [[2 + 2 * l, 3 + 2 * l] for l in range(D - 1, -1, -1)]
    members.append([0, 1] + list(range(6 + 2 * D, len(shapes))))
    offs = [0] * len(shapes)
    buckets = []
    off = 0
    for mem in members:
        start = off
        for i in mem:
            offs[i] = off
            n = 1
            for d in shapes[i]:
                n *= int(d)
            off += n
        buckets.append((start, off))
        off = (off + 3) // 4 * 4
    return offs, buckets, off


_GRAD_VIEWS: dict = {}


def _grad_views(params, depth):
    """(per-parameter (shape, stride, offset) of its view into the flat gradient buffer, buckets,
    total floats), memoised by the parameter shapes: grad_layout and the views' geometry are
    pure functions of them (the host cost of the eager backward, r06)."""
    key = (depth,) + tuple(p.shape for p in params)
    hit = _GRAD_VIEWS.get(key)
    if hit is None:
        offs, buckets, total = grad_layout(key[1:], depth)
        geo = []
        for o, p in zip(offs, params):
            shape = tuple(p.shape)
            stride, acc = [], 1
            for d in reversed(shape):
                stride.append(acc)
                acc *= int(d)
            geo.append((shape, tuple(reversed(stride)), o))
        if len(_GRAD_VIEWS) > 64:
            _GRAD_VIEWS.clear()
        hit = _GRAD_VIEWS[key] = (tuple(geo), buckets, total)
    return hit


# training arena / workspace sizes by (config, N, E, B): pure functions of their key
_ARENA_BYTES: dict = {}
_WS_BYTES: dict = {}


def _memo_bytes(memo, fn, cfg, cfg_tuple, N, E, B):
    key = (cfg_tuple, N, E, B)
    n = memo.get(key)
    if n is None:
        n = fn(ctypes.byref(cfg), N, E, B)
        if n < 0:
            native.check(1)
        if len(memo) > 4096:
            memo.clear()
        memo[key] = n
    return n


def read_status(arena, cfg, N, E, B) -> int:
    """Graph-prep status word (bit0 bad edge index, bit1 bad/unsorted batch, bit2 edges not
    reverse-paired: informational, bit4 the unpaired backward's completion timed out).
    Synchronises."""
    lib = native.load()
    off = lib.cgr_gnn_arena_offset(ctypes.byref(cfg), N, E, B, b"status", 0)
    return int(arena[off:off + 4].view(torch.int32).item())


class GNNFunction(torch.autograd.Function):
    """y[B] = GNN(x, edge_index, edge_attr, batch; params) on the MI355X path."""

    @staticmethod
    def forward(ctx, cfg_tuple, x, edge_index, edge_attr, batch, graph_ptr, num_graphs,
                dropout_ps, seed, rng_counter, training, bucket_hook, *params):
        lib = native.load()
        cfg = make_config(*cfg_tuple)
        N, E, B = int(x.shape[0]), int(edge_index.shape[1]), int(num_graphs)
        dev = x.device
        arena_bytes = _memo_bytes(_ARENA_BYTES, lib.cgr_gnn_arena_bytes, cfg, cfg_tuple, N, E, B)
        arena = torch.empty(arena_bytes, dtype=torch.uint8, device=dev)
        y = torch.empty(B, dtype=torch.float32, device=dev)
        bs = _batch_struct(x, edge_index, edge_attr, batch, graph_ptr, B)
        ptab = _param_table(params)
        dps = _dropout_array(dropout_ps, cfg.depth)
        # CGR_TRAIN_DROPOUT | CGR_TRAIN_FOR_BACKWARD (include/cgr_mpnn3d.h): the backward's
        # weight-gradient operands are prepared only when a gradient is wanted (parameters, or
        # x / edge_attr: the input gradients come after the parameter backward)
        want_bwd = any(ctx.needs_input_grad[12:]) or ctx.needs_input_grad[1] or \
            ctx.needs_input_grad[3]
        flags = (native.TRAIN_DROPOUT if training else 0) | (
            native.TRAIN_FOR_BACKWARD if want_bwd else 0)
        with native.device_guard(dev):
            native.check(lib.cgr_gnn_forward(ctypes.byref(cfg), ptab, ctypes.byref(bs), dps,
                                             ctypes.c_uint64(seed), native.ptr(rng_counter),
                                             flags, native.ptr(arena),
                                             native.ptr(y), native.stream_ptr(dev)))
        if _config.strict:
            raise_on_status(arena, cfg, N, E, B)
        ctx.cfg_tuple = cfg_tuple
        ctx.num_graphs = B
        ctx.dropout_ps = dropout_ps
        ctx.seed = seed
        ctx.training = training
        ctx.flags = flags
        ctx.bucket_hook = bucket_hook
        ctx.save_for_backward(x, edge_index, edge_attr, batch, graph_ptr, arena, *params)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = native.load()
        x, edge_index, edge_attr, batch, graph_ptr, arena, *params = ctx.saved_tensors
        native.raise_device_errors(x.device, clear=False)  # an earlier backward's timeout
        cfg = make_config(*ctx.cfg_tuple)
        N, E, B = int(x.shape[0]), int(edge_index.shape[1]), ctx.num_graphs
        dev = x.device
        ws = torch.empty(_memo_bytes(_WS_BYTES, lib.cgr_gnn_workspace_bytes, cfg, ctx.cfg_tuple,
                                     N, E, B), dtype=torch.uint8, device=dev)
        # one flat gradient buffer in all-reduce bucket order, viewed per parameter
        geo, buckets, total = _grad_views(params, cfg.depth)
        flat = torch.empty(total, dtype=torch.float32, device=dev)
        grads = [flat.as_strided(s, st, o) for s, st, o in geo]
        dy = dy.contiguous().float()
        bs = _batch_struct(x, edge_index, edge_attr, batch, graph_ptr, B)
        hook = ctx.bucket_hook if ctx.bucket_hook is not None else _config.grad_bucket_hook
        # per-bucket ready events (recorded by the native backward) when the hook wants them
        events = None
        if hook is not None and hasattr(hook, "bucket_events"):
            events = hook.bucket_events(dev, len(buckets))
        evtab = None
        if events is not None:
            evtab = (c_void_p * len(events))(*[e.cuda_event for e in events])
        with native.device_guard(dev):
            native.check(lib.cgr_gnn_backward(
                ctypes.byref(cfg), _param_table(params), ctypes.byref(bs),
                _dropout_array(ctx.dropout_ps, cfg.depth), ctypes.c_uint64(ctx.seed),
                ctx.flags, native.ptr(arena), native.ptr(dy), _param_table(grads),
                native.ptr(ws), evtab, native.stream_ptr(dev)))
        dx = dea = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[3]:
            # x.grad / edge_attr.grad (GNN.py:85-86,105-106): from what the backward left in `ws`
            if ctx.needs_input_grad[1]:
                dx = torch.empty(x.shape, dtype=torch.float32, device=dev)
            if ctx.needs_input_grad[3]:
                dea = torch.empty(edge_attr.shape, dtype=torch.float32, device=dev)
            with native.device_guard(dev):
                native.check(lib.cgr_gnn_input_grads(
                    ctypes.byref(cfg), _param_table(params), ctypes.byref(bs), native.ptr(arena),
                    native.ptr(dy), native.ptr(ws),
                    native.ptr(dx) if dx is not None and dx.numel() else None,
                    native.ptr(dea) if dea is not None and dea.numel() else None,
                    native.stream_ptr(dev)))
        if hook is not None:
            # e.g. the RCCL all-reduce of every bucket, each started as soon as its event fires
            # (cgr_mpnn_3D._amd.ddp); must leave the current stream ordered after its work
            hook(flat, buckets, events)
        return (None, dx, None, dea) + (None,) * 8 + tuple(grads)


# predict arena sizes by (config, N, E, B): a pure function of its key (one ctypes call saved per
# call of the single-reaction loop)
_PREDICT_ARENA_BYTES: dict = {}


def gnn_predict(cfg_tuple, x, edge_index, edge_attr, batch, graph_ptr, num_graphs, dropout_ps,
                seed, training, params, rng_counter=None):
    """Forward-only GNN (cgr_gnn_predict): no saved activations.  What GNN.forward runs when no
    gradient is wanted (test.py:100-113 under torch.no_grad()).  The weight images are packed
    into the call's own arena by every call: no cache to go stale when an optimizer (FusedAdam,
    a replayed captured step) updates the parameters through raw pointers, and no buffer shared
    with a predict still running on another stream."""
    lib = native.load()
    cfg = make_config(*cfg_tuple)
    N, E, B = int(x.shape[0]), int(edge_index.shape[1]), int(num_graphs)
    dev = x.device
    key = (cfg_tuple, N, E, B)
    nbytes = _PREDICT_ARENA_BYTES.get(key)
    if nbytes is None:
        nbytes = lib.cgr_gnn_predict_arena_bytes(ctypes.byref(cfg), N, E, B)
        if nbytes < 0:
            native.check(1)
        if len(_PREDICT_ARENA_BYTES) > 4096:
            _PREDICT_ARENA_BYTES.clear()
        _PREDICT_ARENA_BYTES[key] = nbytes
    arena = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    y = torch.empty(B, dtype=torch.float32, device=dev)
    bs = _batch_struct(x, edge_index, edge_attr, batch, graph_ptr, B)
    with native.device_guard(dev):
        native.check(lib.cgr_gnn_predict(
            ctypes.byref(cfg), _param_table(params), ctypes.byref(bs),
            _dropout_array(dropout_ps, cfg.depth), ctypes.c_uint64(seed), native.ptr(rng_counter),
            native.TRAIN_DROPOUT if training else 0, None, native.ptr(arena),
            native.ptr(y), native.stream_ptr(dev)))
    if _config.strict:
        raise_on_status(arena, cfg, N, E, B, predict=True)
    return y


def raise_on_status(arena, cfg, N, E, B, predict=False):
    lib = native.load()
    off = lib.cgr_gnn_arena_offset(ctypes.byref(cfg), N, E, B, b"status", 0)  # same prefix
    st = int(arena[off:off + 4].view(torch.int32).item())
    if st & 1:
        raise IndexError("cgr_mpnn_3D: edge_index holds a node id outside [0, num_nodes)")
    if st & 2:
        raise RuntimeError("cgr_mpnn_3D: batch vector is not sorted / out of range")
    if st & 16:
        raise RuntimeError("cgr_mpnn_3D: the unpaired-edge backward's completion timed out "
                           "(gradients NaN-poisoned, ep_bwd.hpp)")


def gnn_forward(cfg_tuple, x, edge_index, edge_attr, batch, graph_ptr, num_graphs, dropout_ps,
                seed, training, params, bucket_hook=None, rng_counter=None):
    """rng_counter: optional device int64 tensor [1] the forward advances (graph-safe dropout)."""
    return GNNFunction.apply(cfg_tuple, x, edge_index, edge_attr, batch, graph_ptr, num_graphs,
                             dropout_ps, seed, rng_counter, training, bucket_hook, *params)
