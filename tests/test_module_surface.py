"""CPU: the drop-in module keeps the reference's surface (GNN.py:8-145)."""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import act_fn, golden_cases, load_golden

from cgr_mpnn_3D.models.GNN import GNN, DMPNNConv, global_add_pool


@pytest.mark.parametrize("case", [c for c in golden_cases()])
def test_state_dict_keys_shapes_and_seeded_init_match_reference(case):
    z, meta = load_golden(case)
    D, H = meta["depth"], meta["hidden"]
    torch.manual_seed(1000 + len(case))  # the seed make_golden.py used before ref.GNN(...)
    m = GNN(meta["num_node_features"], meta["num_edge_features"], depth=D, hidden_sizes=[H] * D,
            dropout_ps=[meta["eval_dropout"]] * D,
            activation_fn=act_fn(meta["act"]),
            use_learnable_skip=meta["skip"])
    sd = m.state_dict()
    ref_keys = [k[2:] for k in z.files if k.startswith("p_")]
    assert set(sd.keys()) == set(ref_keys)
    for k in ref_keys:
        assert tuple(sd[k].shape) == tuple(z["p_" + k].shape), k
        if not k.startswith("skip_weights"):  # make_golden overwrote sigma after init
            np.testing.assert_array_equal(sd[k].numpy(), z["p_" + k], err_msg=k)


def test_defaults_and_attributes():
    m = GNN(10, 3)
    assert m.depth == 3 and m.hidden_sizes == [300] * 3 and m.dropout_ps == [0.02] * 3
    assert m.activation_fn is F.relu and m.pooling_fn is global_add_pool
    assert not m.use_learnable_skip and not hasattr(m, "skip_weights")
    assert isinstance(m.convs[0], DMPNNConv) and m.convs[0].lin.in_features == 300
    assert m.edge_init.in_features == 13 and m.edge_to_node.in_features == 310
    assert m.ffn.out_features == 1


def test_short_hidden_sizes_raise_index_error_like_reference():
    # BASELINE cfg5 literal: depth 6 with five hidden sizes -> IndexError (GNN.py:59-60)
    with pytest.raises(IndexError):
        GNN(846, 14, depth=6, hidden_sizes=[512] * 5)


def test_cpu_tensors_raise_no_fallback():
    from cgr_mpnn_3D._amd.synth import make_batch

    b = make_batch(2, n_atoms=6, n_bonds=6, n_mace=0).to_torch()
    m = GNN(78, 14, depth=2, hidden_sizes=[16, 16])
    with pytest.raises(RuntimeError, match="GPU"):
        m(b)


def test_global_add_pool_semantics():
    x = torch.arange(12.0).view(6, 2)
    b = torch.tensor([0, 0, 1, 1, 1, 2])
    torch.testing.assert_close(global_add_pool(x, b),
                               torch.tensor([[2.0, 4.0], [18.0, 21.0], [10.0, 11.0]]))
    assert global_add_pool(x, None).shape == (1, 2)


def test_pickle_roundtrip_keeps_class_paths(tmp_path):
    m = GNN(8, 2, depth=2, hidden_sizes=[4, 4], use_learnable_skip=True)
    p = tmp_path / "m.pth"
    torch.save(m, p)
    m2 = torch.load(p, weights_only=False)  # our own file (trainer.py:208 saves full modules)
    assert type(m2).__module__ == "cgr_mpnn_3D.models.GNN"
    for (k1, v1), (k2, v2) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert k1 == k2 and torch.equal(v1, v2)


def test_unpickling_a_reference_style_module_fills_native_state(tmp_path):
    # a checkpoint saved by the reference (trainer.py:208 pickles the whole module) has none of
    # the native path's private state; unpickling into this class must add it
    import torch

    from cgr_mpnn_3D.models.GNN import GNN

    m = GNN(20, 4, depth=2, hidden_sizes=[8, 8])
    for k in ("_grad_bucket_hook", "_cgr_instance"):
        del m.__dict__[k]
    del m._buffers["_cgr_rng_counter"]
    p = tmp_path / "ref_style.pth"
    torch.save(m, p)
    m2 = torch.load(p, weights_only=False)  # our own test file
    assert m2._grad_bucket_hook is None
    assert "_cgr_rng_counter" in m2._buffers and isinstance(m2._cgr_instance, int)
    assert set(m2.state_dict()) == set(m.state_dict())


def test_activation_codes_cover_functions_and_default_modules():
    # the native cgr_activation code per activation_fn (GNN.py:86,127 applies any callable);
    # non-default module parameters and other callables raise: there is no non-native path
    import torch.nn as nn
    from cgr_mpnn_3D._amd import native
    from cgr_mpnn_3D.models.GNN import _activation_code
    fns = {"relu": (F.relu, torch.relu, nn.ReLU()), "silu": (F.silu, nn.SiLU()),
           "gelu": (F.gelu, nn.GELU()), "tanh": (torch.tanh, F.tanh, nn.Tanh()),
           "sigmoid": (torch.sigmoid, F.sigmoid, nn.Sigmoid()), "elu": (F.elu, nn.ELU()),
           "leaky_relu": (F.leaky_relu, nn.LeakyReLU()), "softplus": (F.softplus, nn.Softplus()),
           "mish": (F.mish, nn.Mish()), "selu": (F.selu, torch.selu, nn.SELU())}
    assert set(fns) == set(native.ACT_NAMES)
    for name, cands in fns.items():
        for fn in cands:
            assert _activation_code(fn) == native.ACT_NAMES.index(name), (name, fn)
    for bad in (nn.GELU(approximate="tanh"), nn.LeakyReLU(0.2), nn.ELU(alpha=0.5),
                nn.Softplus(beta=2.0), nn.Softplus(threshold=10.0), torch.abs, lambda t: t):
        with pytest.raises(NotImplementedError):
            _activation_code(bad)
