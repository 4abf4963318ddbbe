"""Batched inference.

The reference evaluates one reaction at a time: ``test.py:85-113`` (DataLoader batch_size 1) and
``cli_tool/activation_energy_predictor.py:71-80`` (per-graph loop, ``batch=None``), both under
``torch.no_grad()`` in eval mode.  Both work unchanged on the native module, whose no-grad calls
take the forward-only path (``cgr_gnn_predict``: no saved activations -- rings of two h and three
a buffers), but each call is still a ~20-launch forward for ~30 atoms.
``predict`` runs that path over large device-collated batches (``GraphStore.collate``), so a whole
test split is a handful of launch sequences.

    store = GraphStore.from_data_list(test_dataset, device)
    y_hat = predict(model, store, batch_size=4096)       # [num_graphs] on the device, in order
"""

from __future__ import annotations

import numpy as np
import torch


@torch.no_grad()
def predict(model, store, ids=None, batch_size: int = 4096) -> torch.Tensor:
    """Eval-mode predictions for graphs ``ids`` (default: all) of a ``GraphStore``."""
    ids = np.arange(store.num_graphs) if ids is None else np.asarray(ids, dtype=np.int64)
    was_training = model.training
    model.eval()
    try:
        outs = [model(store.collate(ids[i:i + batch_size]))
                for i in range(0, ids.size, batch_size)]
    finally:
        model.train(was_training)
    if not outs:
        return torch.empty(0, device=store.device)
    return torch.cat(outs)
