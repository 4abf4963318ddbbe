"""Standalone ``DMPNNConv.forward`` (GNN.py:131-141) on the native kernels, with autograd.

``a`` has ``max(edge_index[1]) + 1`` rows exactly like PyG's inferred scatter size (the conv gets
no node count), which costs one device->host read of that maximum; the fused ``GNN.forward`` path
never calls this.
"""

from __future__ import annotations

import torch

from . import native


class _DMPNNConvFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, edge_index, h, weight, bias, num_nodes, aggregation):
        lib = native.load()
        E, H = int(h.shape[0]), int(h.shape[1])
        dev = h.device
        scratch = torch.empty(lib.cgr_dmpnn_conv_scratch_bytes(num_nodes, E, H), dtype=torch.uint8,
                              device=dev)
        a = torch.empty(num_nodes, H, dtype=torch.float32, device=dev)
        out = torch.empty(E, H, dtype=torch.float32, device=dev)
        with native.device_guard(dev):
            native.check(lib.cgr_dmpnn_conv_forward(
                native.ptr(edge_index), num_nodes, E, native.ptr(h), H, native.ptr(weight),
                native.ptr(bias), native.ptr(a), native.ptr(out), native.ptr(scratch),
                int(aggregation), native.stream_ptr(dev)))
        ctx.save_for_backward(edge_index, h, weight, scratch)
        ctx.num_nodes = num_nodes
        ctx.aggregation = int(aggregation)
        return a, out

    @staticmethod
    def backward(ctx, grad_a, grad_out):
        lib = native.load()
        edge_index, h, weight, scratch = ctx.saved_tensors
        E, H = int(h.shape[0]), int(h.shape[1])
        dev = h.device
        gh = torch.empty_like(h)
        gw = torch.empty_like(weight)
        gb = torch.empty(H, dtype=torch.float32, device=dev)
        ga = None if grad_a is None else grad_a.contiguous().float()
        go = None if grad_out is None else grad_out.contiguous().float()
        with native.device_guard(dev):
            native.check(lib.cgr_dmpnn_conv_backward(
                native.ptr(edge_index), ctx.num_nodes, E, native.ptr(h), H, native.ptr(weight),
                native.ptr(ga), native.ptr(go), native.ptr(gh), native.ptr(gw), native.ptr(gb),
                native.ptr(scratch), ctx.aggregation, native.stream_ptr(dev)))
        return None, gh, gw, gb, None, None


def dmpnn_conv(edge_index, h, weight, bias, aggregation=0):
    """aggregation: 0 "add" (= "sum"), 1 "mean" (include/cgr_mpnn3d.h enum cgr_aggregation)."""
    if not h.is_cuda:
        raise RuntimeError("cgr_mpnn_3D (MI355X): DMPNNConv runs on the GPU only (no CPU fallback)")
    edge_index = edge_index.to(device=h.device, dtype=torch.int64).contiguous()
    if edge_index.shape[1] % 2 or edge_index.shape[1] == 0:
        raise RuntimeError("DMPNNConv: edge_index must hold reverse-edge pairs (GNN.py:136-138)")
    num_nodes = int(edge_index[1].max()) + 1  # PyG's inferred dim_size (x=None at GNN.py:134)
    return _DMPNNConvFunction.apply(edge_index, h.float().contiguous(),
                                    weight.float().contiguous(), bias.float().contiguous(),
                                    num_nodes, aggregation)
