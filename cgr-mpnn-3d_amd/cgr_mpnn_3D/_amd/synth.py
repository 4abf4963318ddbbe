"""Deterministic synthetic Transition1x-shaped reaction batches.

The reference builds one PyG ``Data`` per reaction (``cgr_mpnn_3D/data/ChemDataset.py:81-94``)
and collates them with ``torch_geometric.loader.DataLoader`` (``training/trainer.py:105-118``).
RDKit, MACE and the T1x download are not available here, so benchmarks and parity tests run on
batches of the same *shape* produced by this generator:

* per reaction ``A`` atoms; bonds = a spanning chain ``(i, i+1)`` plus random extra ``(a<b)`` pairs
  up to ``n_bonds``; pairs sorted lexicographically and emitted as ``(a,b),(b,a)`` exactly like
  ``cgr_mpnn_3D/utils/graph_features.py:184-195`` (so ``rev(e) = e ^ 1``);
* ``x`` = 39 reactant atom features (one-hot blocks + mass*0.01) | 39 product-reactant diffs in
  {-1,0,1} | ``n_mace`` Gaussian "MACE" columns (0 for the 2D CGR model);
* ``edge_attr`` = 7 binary bond features | 7 diffs in {-1,0,1} (``graph_features.py:189-192``);
* ``y`` ~ N(80, 20) kcal/mol (demo Ea range, ``cli_tool/files/demo.csv``).

Collation matches PyG ``Batch.from_data_list``: node blocks concatenated, ``edge_index`` offset by
the running node count, ``batch[v]`` = graph id, ``ptr`` = node offsets.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

ATOM_FDIM = 39  # graph_features.py atom_features length (reactant half)
BOND_FDIM = 7  # graph_features.py bond_features length (reactant half)
# one-hot block widths of the 38 categorical reactant columns; col 38 = mass * 0.01
_ATOM_BLOCKS = (11, 7, 5, 5, 6, 3, 1)


@dataclass
class RxnBatch:
    x: np.ndarray  # [N, F] float32
    edge_index: np.ndarray  # [2, E] int64
    edge_attr: np.ndarray  # [E, Fe] float32
    batch: np.ndarray  # [N] int64
    ptr: np.ndarray  # [B+1] int64
    y: np.ndarray  # [B] float32

    @property
    def num_graphs(self) -> int:
        return int(self.ptr.shape[0] - 1)

    def to_torch(self, device=None):
        """Return a duck-typed PyG-Batch-like object holding torch tensors."""
        import torch

        return TorchBatch(
            x=torch.from_numpy(self.x).to(device),
            edge_index=torch.from_numpy(self.edge_index).to(device),
            edge_attr=torch.from_numpy(self.edge_attr).to(device),
            batch=torch.from_numpy(self.batch).to(device),
            ptr=torch.from_numpy(self.ptr).to(device),
            y=torch.from_numpy(self.y).to(device),
        )


class TorchBatch:
    """Minimal stand-in for ``torch_geometric.data.Batch`` (attributes the model reads)."""

    def __init__(self, x, edge_index, edge_attr, batch, ptr=None, y=None):
        self.x = x
        self.edge_index = edge_index
        self.edge_attr = edge_attr
        self.batch = batch
        self.ptr = ptr
        self.y = y

    @property
    def num_graphs(self) -> int:
        if self.ptr is not None:
            return int(self.ptr.numel() - 1)
        if self.batch is None:
            return 1
        return int(self.batch.max().item()) + 1

    def to(self, device):
        def mv(t):
            return None if t is None else t.to(device)

        return TorchBatch(mv(self.x), mv(self.edge_index), mv(self.edge_attr), mv(self.batch),
                          mv(self.ptr), mv(self.y))


def _one_reaction(rng: np.random.Generator, n_atoms: int, n_bonds: int, n_mace: int):
    A = n_atoms
    max_pairs = A * (A - 1) // 2
    n_bonds = max(min(n_bonds, max_pairs), A - 1)
    # spanning chain guarantees connectivity and that the last atom has an (incoming) edge
    chain = set((i, i + 1) for i in range(A - 1))
    extra_needed = n_bonds - len(chain)
    pairs = set(chain)
    if extra_needed > 0:
        # draw candidate pairs in vectorised rounds until enough unique non-chain pairs exist
        while len(pairs) < n_bonds:
            k = max(2 * (n_bonds - len(pairs)), 8)
            a = rng.integers(0, A, size=k)
            b = rng.integers(0, A, size=k)
            for u, v in zip(a.tolist(), b.tolist()):
                if u == v:
                    continue
                p = (u, v) if u < v else (v, u)
                pairs.add(p)
                if len(pairs) >= n_bonds:
                    break
    pairs = sorted(pairs)  # lexicographic (a1 < a2), graph_features.py:184-186
    P = len(pairs)
    ei = np.empty((2, 2 * P), dtype=np.int64)
    pa = np.asarray(pairs, dtype=np.int64).reshape(P, 2)
    ei[0, 0::2] = pa[:, 0]
    ei[1, 0::2] = pa[:, 1]
    ei[0, 1::2] = pa[:, 1]
    ei[1, 1::2] = pa[:, 0]

    # atom features: reactant one-hot blocks + mass, then prod-reac diffs, then MACE
    F = 2 * ATOM_FDIM + n_mace
    x = np.zeros((A, F), dtype=np.float32)
    col = 0
    for w in _ATOM_BLOCKS:
        idx = rng.integers(0, w, size=A)
        x[np.arange(A), col + idx] = 1.0
        col += w
    x[:, 38] = rng.choice(np.array([1.008, 12.011, 14.007, 15.999], dtype=np.float32), size=A) * 0.01
    diff = rng.choice(np.array([-1.0, 0.0, 1.0], dtype=np.float32), size=(A, ATOM_FDIM),
                      p=[0.05, 0.9, 0.05])
    x[:, ATOM_FDIM:2 * ATOM_FDIM] = diff
    if n_mace:
        x[:, 2 * ATOM_FDIM:] = rng.standard_normal((A, n_mace), dtype=np.float32)

    # bond features: one row per undirected bond, duplicated for the reverse edge
    fb = np.zeros((P, 2 * BOND_FDIM), dtype=np.float32)
    fb[:, 0] = 1.0
    btype = rng.integers(1, 5, size=P)
    fb[np.arange(P), btype] = 1.0
    fb[:, 5] = rng.integers(0, 2, size=P)
    fb[:, 6] = rng.integers(0, 2, size=P)
    fb[:, BOND_FDIM:] = rng.choice(np.array([-1.0, 0.0, 1.0], dtype=np.float32),
                                   size=(P, BOND_FDIM), p=[0.1, 0.8, 0.1])
    edge_attr = np.repeat(fb, 2, axis=0)
    return x, ei, edge_attr


def make_batch(num_graphs: int, n_atoms: int = 30, n_bonds: int = 30, n_mace: int = 768,
               seed: int = 1234, n_atoms_jitter: int = 0) -> RxnBatch:
    """Collated batch of ``num_graphs`` synthetic reactions (PyG ``Batch`` layout).

    ``n_atoms_jitter`` > 0 draws per-graph atom counts in ``[n_atoms - j, n_atoms + j]`` (ragged
    batches); bonds scale with the atom count so the edge/atom ratio stays ~2.
    """
    rng = np.random.default_rng(seed)
    xs, eis, eas, bs = [], [], [], []
    ptr = [0]
    off = 0
    for g in range(num_graphs):
        A = n_atoms
        nb = n_bonds
        if n_atoms_jitter:
            A = int(rng.integers(max(2, n_atoms - n_atoms_jitter), n_atoms + n_atoms_jitter + 1))
            nb = max(A - 1, int(round(n_bonds * A / n_atoms)))
        x, ei, ea = _one_reaction(rng, A, nb, n_mace)
        xs.append(x)
        eis.append(ei + off)
        eas.append(ea)
        bs.append(np.full(A, g, dtype=np.int64))
        off += A
        ptr.append(off)
    y = (80.0 + 20.0 * rng.standard_normal(num_graphs)).astype(np.float32)
    return RxnBatch(
        x=np.ascontiguousarray(np.concatenate(xs, 0)),
        edge_index=np.ascontiguousarray(np.concatenate(eis, 1)),
        edge_attr=np.ascontiguousarray(np.concatenate(eas, 0)),
        batch=np.concatenate(bs, 0),
        ptr=np.asarray(ptr, dtype=np.int64),
        y=y,
    )


def make_symmetric_batch(num_graphs: int, n_leaves: int = 3, n_chain: int = 6, n_mace: int = 8,
                         seed: int = 1234) -> RxnBatch:
    """Batch of reactions with symmetric atoms (the explicit hydrogens of one carbon): atom 0
    carries ``n_leaves`` identical leaf atoms (same features, same bond features), then a chain
    of ``n_chain`` atoms.  Every value the model computes for the leaves is then identical, so a
    ``global_max_pool`` column that a leaf wins is a tie (the tie-sharing gradient case)."""
    rng = np.random.default_rng(seed)
    L = n_leaves
    A = 1 + L + n_chain
    pairs = [(0, i) for i in range(1, L + 1)] + [(0, L + 1)] + \
        [(L + 1 + j, L + 2 + j) for j in range(n_chain - 1)]
    P = len(pairs)
    xs, eis, eas, bs, ptr, off = [], [], [], [], [0], 0
    for g in range(num_graphs):
        x, _, ea = _one_reaction(rng, A, A - 1, n_mace)
        assert ea.shape[0] == 2 * P
        x[2:L + 1] = x[1]
        for k in range(1, L):
            ea[2 * k:2 * k + 2] = ea[0:2]
        pa = np.asarray(pairs, dtype=np.int64)
        ei = np.empty((2, 2 * P), dtype=np.int64)
        ei[0, 0::2], ei[1, 0::2] = pa[:, 0], pa[:, 1]
        ei[0, 1::2], ei[1, 1::2] = pa[:, 1], pa[:, 0]
        xs.append(x)
        eis.append(ei + off)
        eas.append(ea)
        bs.append(np.full(A, g, dtype=np.int64))
        off += A
        ptr.append(off)
    y = (80.0 + 20.0 * rng.standard_normal(num_graphs)).astype(np.float32)
    return RxnBatch(x=np.ascontiguousarray(np.concatenate(xs, 0)),
                    edge_index=np.ascontiguousarray(np.concatenate(eis, 1)),
                    edge_attr=np.ascontiguousarray(np.concatenate(eas, 0)),
                    batch=np.concatenate(bs, 0), ptr=np.asarray(ptr, dtype=np.int64), y=y)


# Named workloads of BASELINE.json "configs" (SURVEY.md §8d).
CONFIGS = {
    "cfg1": dict(num_graphs=32, n_atoms=30, n_bonds=30, n_mace=0, depth=2, hidden=128,
                 learnable_skip=False),
    "cfg2": dict(num_graphs=256, n_atoms=30, n_bonds=30, n_mace=768, depth=4, hidden=400,
                 learnable_skip=False),
    "cfg4": dict(num_graphs=256, n_atoms=200, n_bonds=400, n_mace=768, depth=4, hidden=400,
                 learnable_skip=False),
    "cfg5": dict(num_graphs=512, n_atoms=30, n_bonds=30, n_mace=768, depth=6, hidden=512,
                 learnable_skip=True),
    # what train.py users run: its defaults depth 3, hidden 300 (train.py:156-166) at its default
    # batch size 32 (train.py:209), CGR + MACE features
    "train_default": dict(num_graphs=32, n_atoms=30, n_bonds=30, n_mace=768, depth=3, hidden=300,
                          learnable_skip=False),
    # the sweep's other batch sizes (hyperparameter_study/sweep_config.json:12: 16 / 32 / 64) at
    # train.py's default model
    "sweep_b16": dict(num_graphs=16, n_atoms=30, n_bonds=30, n_mace=768, depth=3, hidden=300,
                      learnable_skip=False),
    "sweep_b64": dict(num_graphs=64, n_atoms=30, n_bonds=30, n_mace=768, depth=3, hidden=300,
                      learnable_skip=False),
    # the sweep's depth 5 (sweep_config.json:6) at train.py's default width and batch, and the
    # sweep's largest point: depth 6, hidden 1000, batch 64, learnable skip (:6-7, :12, :15)
    "sweep_d5": dict(num_graphs=32, n_atoms=30, n_bonds=30, n_mace=768, depth=5, hidden=300,
                     learnable_skip=False),
    "sweep_max": dict(num_graphs=64, n_atoms=30, n_bonds=30, n_mace=768, depth=6, hidden=1000,
                      learnable_skip=True),
}
