"""Drop-in ``cgr_mpnn_3D.models.GNN`` for MI355X.

Same module path, class names, constructor arguments, attribute names and ``state_dict`` keys as
the reference (``cgr_mpnn_3D/models/GNN.py:8-145`` of tobjec/CGR-MPNN-3D), so ``train.py``,
``test.py`` and ``hyperparameter_tuning.py`` run unchanged, and the random initialisation for a
given ``torch.manual_seed`` is identical (parameters are created in the reference's order).

What differs is underneath: ``GNN.forward`` is one call into ``libcgr_mpnn3d.so`` (HIP kernels for
gfx950) through ``cgr_mpnn_3D._amd.functional.GNNFunction``; the backward is one more call.  There
is no CPU/PyTorch fallback: CPU tensors or a missing library raise.  ``torch_geometric`` is not
required; PyG ``Batch``/``Data`` objects are accepted by duck typing (``x``, ``edge_index``,
``edge_attr``, ``batch`` and optionally ``ptr`` / ``num_graphs``).

Reference behaviours kept on purpose:
* ``hidden_sizes`` / ``dropout_ps`` shorter than ``depth`` raise ``IndexError`` in ``__init__``
  (``GNN.py:59-60``) / ``forward`` (``GNN.py:100-102``);
* non-uniform hidden sizes are rejected at ``forward`` (the reference fails there on shapes);
* ``batch=None`` pools the whole graph (``global_add_pool(h, None)``), output shape ``[1]``;
* dropout only in training mode (``F.dropout(..., training=self.training)``).
Deliberate deviations: the readout's discarded ``lin`` output (``GNN.py:105``) is not
computed; the scatter size is ``num_nodes`` instead of ``max(dst)+1`` (identical whenever the
batch's last node has an incoming edge; ``CGR_STRICT=1`` raises like the reference otherwise);
dropout masks come from a counter-based RNG keyed by the device's CUDA generator seed
(``torch.cuda.default_generators``, what ``torch.manual_seed`` sets), not ATen's Philox stream.
"""

from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._amd import config as _config
from .._amd import native
from .._amd.functional import gnn_forward, gnn_predict
from .._amd.pool import (aggregation_code, global_add_pool, global_max_pool, global_mean_pool,
                         pooling_code)

__all__ = ["GNN", "DMPNNConv", "global_add_pool", "global_mean_pool", "global_max_pool"]


def _as(t, dtype, dev):
    """``t.to(device=dev, dtype=dtype).contiguous()``, skipping the calls that would return
    ``t`` itself."""
    if t.dtype != dtype or t.device != dev:
        t = t.to(device=dev, dtype=dtype)
    return t if t.is_contiguous() else t.contiguous()


def _activation_code(fn) -> int:
    """The native kernel code (``include/cgr_mpnn3d.h`` ``cgr_activation``) of ``activation_fn``.

    The reference applies any callable (``GNN.py:86,127``); ``train.py:284-292`` offers F.relu /
    F.silu / F.gelu.  Native kernels exist for those and for tanh, sigmoid, ELU, leaky_relu,
    softplus, mish and SELU as functions (``F.*`` / ``torch.*``) or as ``nn`` modules at their
    default parameters; anything else raises (there is no non-native path)."""
    mods = {nn.ReLU: "relu", nn.SiLU: "silu", nn.GELU: "gelu", nn.Tanh: "tanh",
            nn.Sigmoid: "sigmoid", nn.ELU: "elu", nn.LeakyReLU: "leaky_relu",
            nn.Softplus: "softplus", nn.Mish: "mish", nn.SELU: "selu"}
    name = None
    if isinstance(fn, nn.Module):
        name = mods.get(type(fn))
        defaults = {"gelu": ("approximate", "none"), "elu": ("alpha", 1.0),
                    "leaky_relu": ("negative_slope", 0.01), "softplus": ("beta", 1.0)}
        if name in defaults and getattr(fn, defaults[name][0]) != defaults[name][1]:
            name = None
        if name == "softplus" and fn.threshold != 20.0:
            name = None
    else:
        name = getattr(fn, "__name__", "")
    if name in native.ACT_NAMES:
        return native.ACT_NAMES.index(name)
    raise NotImplementedError(
        f"cgr_mpnn_3D (MI355X): activation_fn {fn!r} has no native kernel; supported are relu, "
        "silu, gelu (train.py:284-292), tanh, sigmoid, elu, leaky_relu, softplus, mish, selu "
        "(functions or default-parameter nn modules)")


_UNPAIRED_MSG = (
    "cgr_mpnn_3D: edge_index is not reverse-paired (edge 2k+1 is not the reverse of edge 2k, as "
    "the CGR featuriser emits them, graph_features.py:184-195); results follow the reference's "
    "positional pairing exactly, but the native layer backward then stores every dm row and "
    "completes da = segsum_src(dm) in the last 16 workgroups of each launch (ep_bwd.hpp), several "
    "times slower per layer")


def _warn_if_unpaired(edge_index):
    """A module's first forward (one device sync): warn when edge 2k+1 is not the reverse of edge
    2k.  The reference pairs e with e ^ 1 positionally whatever they hold (flip(view(E/2, 2, H)),
    GNN.py:136-138) and so does the native path, so results stay exact; but the CGR featuriser
    always emits (a, b), (b, a) pairs (graph_features.py:184-195), and the fused layer
    backward's fast form relies on it.  Later batches are covered without a sync: the unpaired
    backward reports itself through the device's error words (cgr_device_errors), which every
    forward reads."""
    import warnings

    e = edge_index
    if e.shape[1] < 2:
        return False
    bad = (e[0, 1::2] != e[1, 0::2]) | (e[1, 1::2] != e[0, 0::2])
    if bool(bad.any()):
        warnings.warn(_UNPAIRED_MSG, RuntimeWarning, stacklevel=3)
        return True
    return False


class GNN(nn.Module):
    """Directed message-passing network over condensed reaction graphs (GNN.py:8-110)."""

    def __init__(
        self,
        num_node_features: int,
        num_edge_features: int,
        depth: int = 3,
        hidden_sizes: list = None,
        dropout_ps: list = None,
        activation_fn=F.relu,
        aggr: str = "add",
        pooling_fn=global_add_pool,
        use_learnable_skip: bool = False,
    ):
        super().__init__()
        self.depth = depth
        self.hidden_sizes = hidden_sizes or [300] * depth
        self.dropout_ps = dropout_ps or [0.02] * depth
        self.activation_fn = activation_fn
        self.pooling_fn = pooling_fn
        self.use_learnable_skip = use_learnable_skip

        # parameter creation order == reference order (same init under torch.manual_seed)
        width0 = self.hidden_sizes[0]
        self.edge_init = nn.Linear(num_node_features + num_edge_features, width0)
        self.convs = nn.ModuleList(
            DMPNNConv(self.hidden_sizes[i], aggr=aggr) for i in range(self.depth))
        width = self.hidden_sizes[-1]
        self.edge_to_node = nn.Linear(num_node_features + width, width)
        self.ffn = nn.Linear(width, 1)
        if self.use_learnable_skip:
            self.skip_weights = nn.ParameterList(
                nn.Parameter(torch.tensor(1.0)) for _ in range(self.depth))
        self._cgr_native_state()

    _cgr_instances = 0  # construction order salts the dropout key (two models, distinct masks)

    def _cgr_native_state(self):
        """State of the native path that the reference module does not have (filled in for
        modules unpickled from a reference checkpoint, test.py:94 / trainer.py:208 save whole
        modules)."""
        if not hasattr(self, "_grad_bucket_hook"):
            # gradient-bucket hook (RCCL all-reduce), set by cgr_mpnn_3D._amd.ddp
            self._grad_bucket_hook = None
        if "_cgr_rng_counter" not in self._buffers:
            # device dropout counter: the native forward advances it, so a HIP-graph-captured
            # training step draws a fresh dropout mask per replay (non-persistent: state_dict
            # keys stay the reference's)
            self.register_buffer("_cgr_rng_counter", torch.zeros(1, dtype=torch.int64),
                                 persistent=False)
        if not hasattr(self, "_cgr_instance"):
            GNN._cgr_instances += 1
            self._cgr_instance = GNN._cgr_instances

    def __setstate__(self, state):
        super().__setstate__(state)
        self._cgr_native_state()

    def _cgr_dropout_seed(self, dev) -> int:
        """Base of the dropout key: the seed of ``dev``'s CUDA generator (what torch.manual_seed
        sets; the reference's F.dropout draws from that generator) mixed with this model's
        construction index.  Reading it consumes nothing, so the CPU RNG stream (DataLoader
        shuffles, random_split) runs exactly as under the reference; the masks vary per forward
        through the device counter the native forward advances."""
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        s = int(torch.cuda.default_generators[idx].initial_seed())
        return (s * 0x9E3779B97F4A7C15 + self._cgr_instance * 0xBF58476D1CE4E5B9) % 2**62

    # -- helpers -------------------------------------------------------------------------------
    def native_parameters(self):
        """Parameters in the C-ABI table order (== reference state_dict order).  Read from the
        submodules' parameter dicts directly (what nn.Module.__getattr__ resolves to, without its
        per-access lookups: this runs on every forward, r06 single-reaction latency)."""
        mods = self._modules
        ei, en, ff = (mods["edge_init"]._parameters, mods["edge_to_node"]._parameters,
                      mods["ffn"]._parameters)
        ps = [ei["weight"], ei["bias"]]
        for conv in mods["convs"]._modules.values():
            lp = conv._modules["lin"]._parameters
            ps += [lp["weight"], lp["bias"]]
        ps += [en["weight"], en["bias"], ff["weight"], ff["bias"]]
        if self.use_learnable_skip:
            ps += list(mods["skip_weights"]._parameters.values())
        return ps

    def _uniform_hidden(self) -> int:
        mods = self._modules
        widths = {mods["edge_init"].out_features, mods["edge_to_node"].out_features}
        widths |= {conv._modules["lin"].out_features for conv in mods["convs"]._modules.values()}
        if len(widths) != 1:
            raise RuntimeError(
                f"GNN: hidden sizes {sorted(widths)} differ; the D-MPNN skip connection "
                "(GNN.py:94-97) needs one uniform hidden size")
        return widths.pop()

    # -- forward -------------------------------------------------------------------------------
    def forward(self, data):
        x, edge_index, edge_attr, batch = data.x, data.edge_index, data.edge_attr, data.batch
        if not x.is_cuda:
            raise RuntimeError(
                "cgr_mpnn_3D (MI355X) runs on the GPU only: move the model and the batch to "
                "'cuda' (there is no CPU fallback)")
        pool = pooling_code(self.pooling_fn)
        aggrs = {aggregation_code(conv.aggr) for conv in self._modules["convs"]._modules.values()}
        if len(aggrs) != 1:
            raise NotImplementedError("cgr_mpnn_3D (MI355X): one aggr for every DMPNNConv")
        aggr = aggrs.pop()
        act = _activation_code(self.activation_fn)
        H = self._uniform_hidden()
        drop = [float(self.dropout_ps[l]) for l in range(self.depth)]  # IndexError like GNN.py:101

        dev = x.device
        # dtype / device / layout conversions only where needed (each .to().contiguous() pair
        # costs ~2.5 us of dispatch even when it returns its input)
        x = _as(x, torch.float32, dev)
        edge_index = _as(edge_index, torch.int64, dev)
        F_ = x.shape[1]
        Fe = self.edge_init.in_features - F_
        if edge_attr is None:
            edge_attr = x.new_zeros((edge_index.shape[1], 0))
        edge_attr = _as(edge_attr, torch.float32, dev)
        if edge_attr.dim() != 2 or edge_attr.shape[1] != Fe:
            raise RuntimeError(
                f"GNN: edge_init expects {self.edge_init.in_features} = num_node_features + "
                f"num_edge_features inputs, got x[:, {F_}] and edge_attr {tuple(edge_attr.shape)}")
        if self.edge_to_node.in_features != F_ + H:
            raise RuntimeError("GNN: edge_to_node input width does not match x")
        if edge_index.shape[1] % 2:
            raise RuntimeError("GNN: edge_index must hold reverse-edge pairs (GNN.py:136-138)")

        graph_ptr = None
        if batch is None:
            num_graphs = 1
        else:
            batch = _as(batch, torch.int64, dev)
            ptr = getattr(data, "ptr", None)
            if ptr is not None and ptr.numel() >= 2 and ptr.is_cuda:
                graph_ptr = _as(ptr, torch.int64, ptr.device)
                num_graphs = graph_ptr.numel() - 1
            else:
                ng = getattr(data, "num_graphs", None)
                num_graphs = int(ng) if ng is not None else int(batch.max()) + 1
        if _config.strict and int(edge_index[1].max()) + 1 != x.shape[0]:
            # the reference's cat([x, s]) (GNN.py:106) fails when the last node has no in-edge
            raise RuntimeError(
                "Sizes of tensors must match: scatter size max(edge_index[1])+1 != num_nodes")

        # kernel-reported conditions (no sync): an unpaired backward's completion that timed out
        # raises here; an unpaired batch seen by any earlier backward warns once per module
        if native.raise_device_errors(dev) & native.DEVERR_UNPAIRED_SEEN and \
                not getattr(self, "_cgr_unpaired_warned", False):
            import warnings

            self._cgr_unpaired_warned = True
            warnings.warn(_UNPAIRED_MSG, RuntimeWarning, stacklevel=2)
        if not getattr(self, "_cgr_pairing_checked", False) and \
                not torch.cuda.is_current_stream_capturing():
            self._cgr_pairing_checked = True
            if not getattr(self, "_cgr_unpaired_warned", False) and _warn_if_unpaired(edge_index):
                self._cgr_unpaired_warned = True

        params = self.native_parameters()
        want_grad = x.requires_grad or edge_attr.requires_grad
        for i, p in enumerate(params):
            if p.dtype != torch.float32 or not p.is_cuda:
                raise RuntimeError("cgr_mpnn_3D (MI355X): parameters must be fp32 CUDA tensors")
            if not p.is_contiguous():
                params[i] = p.contiguous()
            want_grad = want_grad or p.requires_grad
        training = self.training and any(p > 0 for p in drop)
        seed = self._cgr_dropout_seed(dev) if training else 0
        counter = self._cgr_rng_counter
        if counter.device != dev:
            counter = self._cgr_rng_counter = counter.to(dev)
        cfg = (F_, Fe, H, self.depth, act, self.use_learnable_skip, aggr, pool)
        if not (torch.is_grad_enabled() and want_grad):
            # no gradient wanted (test.py / the CLI run under torch.no_grad()): the forward-only
            # path, no saved activations
            # (no autograd here: the raw parameters' data pointers, no detach)
            return gnn_predict(cfg, x, edge_index, edge_attr, batch, graph_ptr, num_graphs, drop,
                               seed, training, params, rng_counter=counter)
        return gnn_forward(cfg, x, edge_index, edge_attr, batch, graph_ptr, num_graphs, drop,
                           seed, training, params, self._grad_bucket_hook, rng_counter=counter)


class DMPNNConv(nn.Module):
    """One directed message-passing step (GNN.py:113-145).

    ``forward(edge_index, edge_attr) -> (a, h')`` with ``a[v] = sum_{dst(e)=v} edge_attr[e]`` and
    ``h'[e] = lin(a[src(e)] - edge_attr[e ^ 1])``.  Runs on the native segmented-sum + gathered
    MFMA GEMM kernels (``cgr_dmpnn_conv_forward``/``_backward``).  ``GNN.forward`` does not call
    it: the fused path inlines it.
    """

    def __init__(self, hidden_size: int, aggr="add"):
        super().__init__()
        self.aggr = aggr
        self.lin = nn.Linear(hidden_size, hidden_size)

    def forward(self, edge_index, edge_attr):
        from .._amd.conv import dmpnn_conv

        return dmpnn_conv(edge_index, edge_attr, self.lin.weight, self.lin.bias,
                          aggregation_code(self.aggr))

    def message(self, edge_attr):
        return edge_attr
