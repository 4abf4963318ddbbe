"""ORACLE (test infrastructure only) - numpy restatement of PyG batch collation.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the *checker* / CPU baseline of the on-device collation
(``cgr_collate``, ``cgr_mpnn_3D/_amd/data.py``).

The reference collates per-reaction ``Data`` objects (``cgr_mpnn_3D/data/ChemDataset.py:81-94``)
with ``torch_geometric.loader.DataLoader`` (``cgr_mpnn_3D/training/trainer.py:105-118``), i.e.
``Batch.from_data_list``.  PyG is not installed here; its documented collation
semantics for these fields are restated: ``x`` / ``edge_attr`` / ``y`` concatenated in list order,
``edge_index`` offset by the number of nodes of the preceding graphs (``__inc__`` of
``edge_index`` = ``num_nodes``), ``batch[v]`` = position of v's graph in the list, ``ptr`` = the
cumulative node counts.  Integer and byte work: the device result must match bit for bit.
"""

from __future__ import annotations

import numpy as np


def collate(ids, x, edge_index, edge_attr, y, node_ptr, edge_ptr):
    """Batch.from_data_list of graphs ``ids`` of a store in collated layout (global node ids)."""
    ids = np.asarray(ids, dtype=np.int64).reshape(-1)
    xs, eis, eas, bs, ys = [], [], [], [], []
    ptr = [0]
    for pos, g in enumerate(ids.tolist()):
        n0, n1 = int(node_ptr[g]), int(node_ptr[g + 1])
        e0, e1 = int(edge_ptr[g]), int(edge_ptr[g + 1])
        xs.append(x[n0:n1])
        eis.append(edge_index[:, e0:e1] - n0 + ptr[-1])  # local ids + running node count
        eas.append(edge_attr[e0:e1])
        bs.append(np.full(n1 - n0, pos, dtype=np.int64))
        if y is not None:
            ys.append(y[g])
        ptr.append(ptr[-1] + (n1 - n0))
    F = x.shape[1]
    Fe = edge_attr.shape[1]
    return dict(
        x=np.concatenate(xs, 0) if xs else np.zeros((0, F), np.float32),
        edge_index=np.concatenate(eis, 1) if eis else np.zeros((2, 0), np.int64),
        edge_attr=np.concatenate(eas, 0) if eas else np.zeros((0, Fe), np.float32),
        batch=np.concatenate(bs, 0) if bs else np.zeros(0, np.int64),
        ptr=np.asarray(ptr, dtype=np.int64),
        y=np.asarray(ys, dtype=np.float32) if y is not None else None,
    )
