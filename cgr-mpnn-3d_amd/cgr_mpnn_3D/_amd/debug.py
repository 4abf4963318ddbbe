"""Introspection helpers (tests / profiling): run the native forward with a caller-visible arena
and view its saved buffers.  Not used by the model itself."""

from __future__ import annotations

import ctypes

import torch

from . import native
from .functional import _batch_struct, _dropout_array, _param_table, make_config


class ArenaRun:
    def __init__(self, cfg_tuple, x, edge_index, edge_attr, batch, graph_ptr, num_graphs, params,
                 dropout_ps=None, seed=0, training=False, prepare_backward=True):
        lib = native.load()
        self.cfg = make_config(*cfg_tuple)
        self.N, self.E, self.B = int(x.shape[0]), int(edge_index.shape[1]), int(num_graphs)
        self.H = self.cfg.hidden
        self.Hp = (self.H + 3) // 4 * 4
        dev = x.device
        nbytes = lib.cgr_gnn_arena_bytes(ctypes.byref(self.cfg), self.N, self.E, self.B)
        self.arena = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self.y = torch.empty(self.B, dtype=torch.float32, device=dev)
        self._keep = (x, edge_index, edge_attr, batch, graph_ptr, params)
        self.bs = _batch_struct(x, edge_index, edge_attr, batch, graph_ptr, self.B)
        self.dropout_ps, self.seed, self.training = dropout_ps, seed, training
        # prepared for the backward (this helper runs it), as a training step's forward is
        self.flags = (native.TRAIN_DROPOUT if training else 0) | (
            native.TRAIN_FOR_BACKWARD if prepare_backward else 0)
        with native.device_guard(dev):
            native.check(lib.cgr_gnn_forward(
                ctypes.byref(self.cfg), _param_table(params), ctypes.byref(self.bs),
                _dropout_array(dropout_ps, self.cfg.depth), ctypes.c_uint64(seed), None,
                self.flags, native.ptr(self.arena), native.ptr(self.y),
                native.stream_ptr(dev)))

    def offset(self, name, index=0):
        lib = native.load()
        return lib.cgr_gnn_arena_offset(ctypes.byref(self.cfg), self.N, self.E, self.B,
                                        name.encode(), index)

    def ints(self, name, count):
        off = self.offset(name)
        assert off >= 0, name
        return self.arena[off:off + 4 * count].view(torch.int32)

    def floats(self, name, rows, index=0, cols=None):
        off = self.offset(name, index)
        assert off >= 0, (name, index)
        cols = self.Hp if cols is None else cols
        t = self.arena[off:off + 4 * rows * cols].view(torch.float32).view(rows, cols)
        return t[:, :self.H] if cols == self.Hp else t

    def backward(self, dy, params):
        lib = native.load()
        dev = dy.device
        ws = torch.empty(lib.cgr_gnn_workspace_bytes(ctypes.byref(self.cfg), self.N, self.E,
                                                     self.B), dtype=torch.uint8, device=dev)
        grads = [torch.empty_like(p) for p in params]
        self.ws = ws
        with native.device_guard(dev):
            native.check(lib.cgr_gnn_backward(
                ctypes.byref(self.cfg), _param_table(params), ctypes.byref(self.bs),
                _dropout_array(self.dropout_ps, self.cfg.depth), ctypes.c_uint64(self.seed),
                self.flags, native.ptr(self.arena), native.ptr(dy.contiguous()),
                _param_table(grads), native.ptr(ws), None, native.stream_ptr(dev)))
        return grads

    def input_grads(self, dy, params, ws):
        """cgr_gnn_input_grads on this arena with workspace `ws` -> (dx, dedge_attr)."""
        lib = native.load()
        dev = dy.device
        F_ = self.cfg.num_node_features
        Fe = self.cfg.num_edge_features
        dx = torch.empty(self.N, F_, device=dev)
        de = torch.empty(self.E, Fe, device=dev) if Fe else None
        with native.device_guard(dev):
            native.check(lib.cgr_gnn_input_grads(
                ctypes.byref(self.cfg), _param_table(params), ctypes.byref(self.bs),
                native.ptr(self.arena), native.ptr(dy.contiguous()), native.ptr(ws),
                native.ptr(dx), native.ptr(de), native.stream_ptr(dev)))
        return dx, de
