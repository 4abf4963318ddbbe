"""CPU (gloo, world_size 2): data-parallel path = graph-sharded batch + SUM all-reduce of the flat
gradient bucket.  The per-rank compute here is the oracle (CPU); on the GPU box the same hook is
called by the native backward with RCCL."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cgr_mpnn_3D._amd.ddp import install_grad_allreduce, shard_batch, shard_ranges
from cgr_mpnn_3D._amd.synth import make_batch


def test_shard_ranges_balanced_contiguous():
    rng = np.random.default_rng(0)
    edges = rng.integers(20, 200, size=256)
    for world in (1, 2, 3, 4, 8):
        rs = shard_ranges(edges, world)
        assert rs[0][0] == 0 and rs[-1][1] == 256
        assert all(a < b for a, b in rs) and all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
        loads = [edges[a:b].sum() for a, b in rs]
        assert max(loads) - min(loads) <= 2 * edges.max()
    with pytest.raises(ValueError):
        shard_ranges(edges[:3], 4)


def test_shard_batch_is_a_valid_collated_batch():
    b = make_batch(10, n_atoms=12, n_bonds=14, n_mace=0, seed=2, n_atoms_jitter=5)
    parts = [shard_batch(b, r, 3) for r in range(3)]
    assert sum(p.num_graphs for p in parts) == 10
    assert sum(p.x.shape[0] for p in parts) == b.x.shape[0]
    assert sum(p.edge_index.shape[1] for p in parts) == b.edge_index.shape[1]
    for p in parts:
        N = p.x.shape[0]
        assert p.edge_index.min() >= 0 and p.edge_index.max() < N
        assert p.ptr[0] == 0 and p.ptr[-1] == N
        assert np.array_equal(p.batch, np.repeat(np.arange(p.num_graphs), np.diff(p.ptr)))
        # reverse pairs preserved
        assert np.array_equal(p.edge_index[0, 0::2], p.edge_index[1, 1::2])
    np.testing.assert_array_equal(np.concatenate([p.y for p in parts]), b.y)


def test_grad_layout_buckets_cover_every_parameter_once():
    from cgr_mpnn_3D._amd.functional import grad_layout

    for D, skip in ((1, False), (4, False), (6, True)):
        H, F, Fe = 8, 10, 3
        shapes = [(H, F + Fe), (H,)]
        for _ in range(D):
            shapes += [(H, H), (H,)]
        shapes += [(H, F + H), (H,), (1, H), (1,)]
        shapes += [()] * (D if skip else 0)
        offs, buckets, total = grad_layout(shapes, D)
        assert len(buckets) == D + 2  # CGR_GRAD_BUCKETS(depth)
        cover = np.zeros(total, np.int64)
        for o, sh in zip(offs, shapes):
            n = int(np.prod(sh)) if sh else 1
            cover[o:o + n] += 1
        assert cover.max() == 1  # disjoint
        inb = np.zeros(total, np.int64)
        for a, b in buckets:
            assert a % 4 == 0 and a <= b <= total
            inb[a:b] += 1
        assert np.array_equal(inb, cover)  # buckets hold exactly the parameters
        # readiness order: bucket 0 = edge_to_node + ffn, then layers D-1 .. 0, last edge_init
        assert buckets[0][0] == offs[2 + 2 * D] == 0
        for k in range(D):
            l = D - 1 - k
            assert buckets[1 + k] == (offs[2 + 2 * l], offs[3 + 2 * l] + H)
        assert buckets[-1][0] == offs[0]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Model:
    _grad_bucket_hook = None


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import dmpnn_numpy as on
        from oracle.dmpnn_torch import random_state_dict

        full = make_batch(8, n_atoms=10, n_bonds=12, n_mace=4, seed=5)
        sd = {k: v.numpy().astype(np.float64)
              for k, v in random_state_dict(full.x.shape[1], 14, 8, 2, seed=3).items()}
        keys = list(sd)
        part = shard_batch(full, rank, world)
        _, _, g = on.loss_and_grads(sd, part.x, part.edge_index, part.edge_attr, part.batch,
                                    part.y, 2, "relu", False, num_graphs=part.num_graphs)
        from cgr_mpnn_3D._amd.functional import grad_layout

        # the native backward's flat buffer: bucket order, 16-byte aligned buckets
        offs, buckets, total = grad_layout([sd[k].shape for k in keys], 2)
        flat = torch.zeros(total, dtype=torch.float64)
        for k, o in zip(keys, offs):
            flat[o:o + g[k].size] = torch.from_numpy(np.ravel(g[k]))
        m = install_grad_allreduce(_Model())
        m._grad_bucket_hook(flat, buckets, None)  # what the native backward calls (no events)
        if rank == 0:
            _, _, gf = on.loss_and_grads(sd, full.x, full.edge_index, full.edge_attr, full.batch,
                                         full.y, 2, "relu", False, num_graphs=full.num_graphs)
            ref = np.zeros(total)
            for k, o in zip(keys, offs):
                ref[o:o + gf[k].size] = np.ravel(gf[k])
            q.put(float(np.abs(flat.numpy() - ref).max() / np.abs(ref).max()))
    finally:
        dist.destroy_process_group()


def test_sum_allreduce_of_shard_gradients_equals_global_batch_gradient():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    err = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert err < 1e-12


def test_teardown_warns_when_captured_collectives_may_outlive_the_group():
    """ddp.teardown's precondition (drop every graph that recorded a collective first) is a
    checked argument: a hook that recorded collectives into a capture, torn down without
    graphs_released=True, warns before the communicator is destroyed."""
    import warnings

    from cgr_mpnn_3D._amd.ddp import teardown

    class _M:
        pass

    for released, expect in ((False, True), (True, False)):
        store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
        dist.init_process_group("gloo", store=store, rank=0, world_size=1)
        m = install_grad_allreduce(_M())
        m._grad_bucket_hook.captured = 3  # as after a captured backward
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            teardown(m, graphs_released=released)
        hits = [x for x in w if "graphs_released" in str(x.message)]
        assert bool(hits) == expect
        assert not dist.is_initialized() and m._grad_bucket_hook is None
