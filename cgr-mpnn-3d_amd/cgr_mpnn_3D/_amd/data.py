"""Device-resident reaction-graph store + on-device collation.

The reference loads every reaction as a PyG ``Data`` (``cgr_mpnn_3D/data/ChemDataset.py:81-94``)
and collates each step's batch on the host with ``torch_geometric.loader.DataLoader``
(``cgr_mpnn_3D/training/trainer.py:105-118``), then copies it to the GPU.  At ~1.4 ms per
training step on one MI355X that host path (collating 256 graphs + a 26 MB H2D copy) would cost
more than the step itself.  Here the whole dataset (T1x: ~10k reactions, ~1 GB fp32 with the
768-wide MACE block) is uploaded once, and each batch is collated by one kernel
(``cgr_collate``) into exactly the ``Batch.from_data_list`` layout ``GNN.forward`` reads.

    store = GraphStore.from_data_list(list_of_pyg_data, device)   # or from_batch(collated)
    for ids in sampler:                                             # host int indices
        batch = store.collate(ids)                                  # device TorchBatch
        loss = loss_fn(model(batch), batch.y)

``collate`` needs the output sizes for allocation; they come from the host copy of the per-graph
node/edge counts, so there is no device sync.  There is no CPU fallback.
"""

from __future__ import annotations

import numpy as np
import torch

from . import native
from .synth import RxnBatch, TorchBatch


class GraphStore:
    def __init__(self, x, edge_index, edge_attr, y, node_ptr, edge_ptr, device):
        """All arrays in collated (PyG ``Batch``) layout on the host (numpy): x [N, F] float32,
        edge_index [2, E] int64 with global node ids, edge_attr [E, Fe] float32, y [G] float32
        or None, node_ptr / edge_ptr [G+1] int64."""
        dev = torch.device(device)
        if dev.type != "cuda":
            raise RuntimeError("GraphStore lives on the GPU (no CPU fallback)")
        self.node_ptr_h = np.asarray(node_ptr, dtype=np.int64)
        self.edge_ptr_h = np.asarray(edge_ptr, dtype=np.int64)
        self.num_graphs = int(self.node_ptr_h.shape[0] - 1)
        self.F = int(x.shape[1])
        self.Fe = int(edge_attr.shape[1]) if edge_attr is not None else 0
        self.device = dev
        self.x = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(dev)
        self.edge_index = torch.from_numpy(
            np.ascontiguousarray(edge_index, dtype=np.int64)).to(dev)
        self.edge_attr = (torch.from_numpy(np.ascontiguousarray(edge_attr, dtype=np.float32))
                          .to(dev) if self.Fe else None)
        self.y = (torch.from_numpy(np.ascontiguousarray(y, dtype=np.float32)).to(dev)
                  if y is not None else None)
        self.node_ptr = torch.from_numpy(self.node_ptr_h).to(dev)
        self.edge_ptr = torch.from_numpy(self.edge_ptr_h).to(dev)
        self._ncount = np.diff(self.node_ptr_h)
        self._ecount = np.diff(self.edge_ptr_h)
        self._lib = native.load()

    # -- construction ------------------------------------------------------------------------
    @classmethod
    def from_batch(cls, b: RxnBatch, device):
        """From one collated batch holding the whole dataset (edges grouped by graph, as PyG
        collation leaves them)."""
        src_graph = b.batch[b.edge_index[0]]
        if src_graph.size and np.any(np.diff(src_graph) < 0):
            raise ValueError("edges must be grouped by graph (PyG collation order)")
        ecount = np.bincount(src_graph, minlength=b.num_graphs)
        edge_ptr = np.concatenate([[0], np.cumsum(ecount)]).astype(np.int64)
        return cls(b.x, b.edge_index, b.edge_attr, b.y, b.ptr, edge_ptr, device)

    @classmethod
    def from_data_list(cls, data_list, device):
        """From per-reaction PyG-``Data``-like objects (attributes x, edge_index, edge_attr, y;
        torch tensors or numpy arrays), e.g. ``ChemDataset``'s items."""
        def np_(t):
            if t is None:
                return None
            return t.detach().cpu().numpy() if hasattr(t, "detach") else np.asarray(t)

        xs, eis, eas, ys = [], [], [], []
        nptr, eptr = [0], [0]
        for d in data_list:
            x = np_(d.x).astype(np.float32)
            ei = np_(d.edge_index).astype(np.int64)
            ea = np_(getattr(d, "edge_attr", None))
            xs.append(x)
            eis.append(ei + nptr[-1])
            eas.append(ea.astype(np.float32) if ea is not None
                       else np.zeros((ei.shape[1], 0), np.float32))
            y = np_(getattr(d, "y", None))
            ys.append(np.float32(np.asarray(y).reshape(-1)[0]) if y is not None else np.nan)
            nptr.append(nptr[-1] + x.shape[0])
            eptr.append(eptr[-1] + ei.shape[1])
        y = np.asarray(ys, dtype=np.float32)
        return cls(np.concatenate(xs, 0), np.concatenate(eis, 1), np.concatenate(eas, 0),
                   None if np.isnan(y).all() else y, np.asarray(nptr), np.asarray(eptr), device)

    # -- collation ---------------------------------------------------------------------------
    def batch_sizes(self, ids: np.ndarray) -> tuple[int, int]:
        return int(self._ncount[ids].sum()), int(self._ecount[ids].sum())

    def collate(self, ids, stream=None) -> TorchBatch:
        """Batch of graphs ``ids`` (host ints, any order, repeats allowed) in
        ``Batch.from_data_list`` layout, built on the device by one kernel."""
        ids = np.ascontiguousarray(np.asarray(ids, dtype=np.int64).reshape(-1))
        if ids.size and (ids.min() < 0 or ids.max() >= self.num_graphs):
            raise IndexError(f"graph id out of range [0, {self.num_graphs})")
        B = int(ids.size)
        N, E = self.batch_sizes(ids)
        dev = self.device
        gid = torch.from_numpy(ids).to(dev, non_blocking=False)
        x = torch.empty((N, self.F), dtype=torch.float32, device=dev)
        ei = torch.empty((2, E), dtype=torch.int64, device=dev)
        ea = torch.empty((E, self.Fe), dtype=torch.float32, device=dev)
        bt = torch.empty(N, dtype=torch.int64, device=dev)
        ptr = torch.empty(B + 1, dtype=torch.int64, device=dev)
        y = torch.empty(B, dtype=torch.float32, device=dev) if self.y is not None else None
        if B:
            with native.device_guard(dev):
                native.check(self._lib.cgr_collate(
                    native.ptr(gid), B, native.ptr(self.node_ptr), native.ptr(self.edge_ptr),
                    native.ptr(self.x), self.F, native.ptr(self.edge_index),
                    int(self.edge_index.shape[1]), native.ptr(self.edge_attr), self.Fe,
                    native.ptr(self.y), native.ptr(x), native.ptr(ei), E, native.ptr(ea),
                    native.ptr(bt), native.ptr(ptr), native.ptr(y),
                    stream if stream is not None else native.stream_ptr(dev)))
        else:
            ptr.zero_()
        out = TorchBatch(x=x, edge_index=ei, edge_attr=ea, batch=bt, ptr=ptr, y=y)
        out._ids = gid  # keep the id buffer alive until the kernel has run
        return out
