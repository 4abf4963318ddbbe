"""ORACLE (test infrastructure only) - numpy float64 restatement of the CGR-MPNN-3D D-MPNN.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the *checker*.  The product path (``cgr_mpnn_3D.models.GNN`` -> C-ABI ->
HIP kernels) never calls into ``oracle/``.

Pinning: the forward and every parameter gradient of this restatement are checked against golden
vectors produced by running the reference ``cgr_mpnn_3D/models/GNN.py`` itself
(``tests/golden/make_golden.py``; ``tests/test_oracle_golden.py``).

What is restated (reference = tobjec/CGR-MPNN-3D @ 2025-02-27):

* ``graph_prep``          index bookkeeping the HIP path uses: stable dst-sort ``perm``,
                          ``dst_ptr`` (bincount+cumsum), ``rev_s = perm^-1[perm ^ 1]`` (the
                          ``flip(view(E/2,2,H))`` of ``GNN.py:136-138`` in sorted space), src-CSR
                          over sorted positions, graph ``ptr`` from ``batch``.
* ``forward``             ``GNN.forward`` ``GNN.py:76-110`` with PyG's sum-scatter
                          (``propagate`` ``GNN.py:134`` / ``global_add_pool`` ``GNN.py:110``)
                          restated as a sparse incidence product, ``dim_size = N``.
* ``backward``            hand-derived reverse mode of the above, the exact
                          sequence the HIP backward kernels implement; with ``inputs_out`` also
                          the gradients w.r.t. ``x`` (through ``x[row]``, ``GNN.py:85-86``, and
                          ``cat([x, s])``, ``GNN.py:105-106``) and ``edge_attr`` (``GNN.py:86``),
                          pinned by the goldens' ``gin_*`` arrays (reference autograd).
"""

from __future__ import annotations

import numpy as np

try:  # scipy is only used for speed (sparse scatter) and erf
    import scipy.sparse as _sp
    from scipy.special import erf as _erf
except Exception:  # pragma: no cover
    _sp = None
    _erf = None

ACT_CODES = {"relu": 0, "silu": 1, "gelu": 2, "tanh": 3, "sigmoid": 4, "elu": 5, "leaky_relu": 6,
             "softplus": 7, "mish": 8, "selu": 9}
_SELU_ALPHA, _SELU_SCALE = 1.6732632423543772848170429916717, 1.0507009873554804934193349852946


# ----------------------------------------------------------------------------------------------
# activations (train.py:284-292: F.relu / F.silu / F.gelu(approximate='none'))
# ----------------------------------------------------------------------------------------------
def act_fwd(z: np.ndarray, act: str) -> np.ndarray:
    if act == "relu":
        return np.maximum(z, 0.0)
    if act == "silu":
        return z / (1.0 + np.exp(-z))
    if act == "gelu":
        return 0.5 * z * (1.0 + _erf(z / np.sqrt(2.0)))
    # further elementwise activations at torch's default parameters (torch.nn.functional)
    if act == "tanh":
        return np.tanh(z)
    if act == "sigmoid":
        return 1.0 / (1.0 + np.exp(-z))
    if act == "elu":
        return np.where(z > 0, z, np.expm1(np.minimum(z, 0.0)))
    if act == "leaky_relu":
        return np.where(z > 0, z, 0.01 * z)
    if act == "softplus":
        return np.where(z > 20.0, z, np.log1p(np.exp(np.minimum(z, 20.0))))
    if act == "mish":
        return z * np.tanh(act_fwd(z, "softplus"))
    if act == "selu":
        return _SELU_SCALE * np.where(z > 0, z, _SELU_ALPHA * np.expm1(np.minimum(z, 0.0)))
    raise ValueError(act)


def act_grad(z: np.ndarray, act: str) -> np.ndarray:
    """d act(z) / dz (ReLU: 0 at z == 0, like ATen's threshold_backward)."""
    if act == "relu":
        return (z > 0).astype(z.dtype)
    if act == "silu":
        s = 1.0 / (1.0 + np.exp(-z))
        return s * (1.0 + z * (1.0 - s))
    if act == "gelu":
        cdf = 0.5 * (1.0 + _erf(z / np.sqrt(2.0)))
        pdf = np.exp(-0.5 * z * z) / np.sqrt(2.0 * np.pi)
        return cdf + z * pdf
    if act == "tanh":
        return 1.0 - np.tanh(z) ** 2
    if act == "sigmoid":
        s = 1.0 / (1.0 + np.exp(-z))
        return s * (1.0 - s)
    if act == "elu":  # ATen elu_backward: x > 0 ? 1 : alpha * exp(x)
        return np.where(z > 0, 1.0, np.exp(np.minimum(z, 0.0)))
    if act == "leaky_relu":
        return np.where(z > 0, 1.0, 0.01).astype(z.dtype)
    if act == "softplus":
        return np.where(z > 20.0, 1.0, 1.0 / (1.0 + np.exp(-z)))
    if act == "mish":
        t = np.tanh(act_fwd(z, "softplus"))
        s = 1.0 / (1.0 + np.exp(-z))
        return t + z * s * (1.0 - t * t)
    if act == "selu":
        return _SELU_SCALE * np.where(z > 0, 1.0, _SELU_ALPHA * np.exp(np.minimum(z, 0.0)))
    raise ValueError(act)


# ----------------------------------------------------------------------------------------------
# index bookkeeping (bit-exact contract for the HIP graph-prep kernels)
# ----------------------------------------------------------------------------------------------
def graph_prep(edge_index: np.ndarray, num_nodes: int, batch: np.ndarray | None = None,
               num_graphs: int | None = None) -> dict:
    src = np.asarray(edge_index[0], dtype=np.int64)
    dst = np.asarray(edge_index[1], dtype=np.int64)
    E = src.shape[0]
    perm = np.argsort(dst, kind="stable").astype(np.int64)  # sorted position -> original edge
    inv = np.empty_like(perm)
    inv[perm] = np.arange(E, dtype=np.int64)
    dst_s = dst[perm]
    src_s = src[perm]
    rev_s = inv[perm ^ 1] if E else perm.copy()  # GNN.py:136-138: reverse of edge e is e ^ 1
    dst_ptr = np.zeros(num_nodes + 1, dtype=np.int64)
    dst_ptr[1:] = np.cumsum(np.bincount(dst, minlength=num_nodes)[:num_nodes])
    src_list = np.argsort(src_s, kind="stable").astype(np.int64)  # sorted positions by src
    src_ptr = np.zeros(num_nodes + 1, dtype=np.int64)
    src_ptr[1:] = np.cumsum(np.bincount(src_s, minlength=num_nodes)[:num_nodes])
    out = dict(perm=perm, dst_s=dst_s, src_s=src_s, rev_s=rev_s, dst_ptr=dst_ptr,
               src_ptr=src_ptr, src_list=src_list)
    if batch is None:
        out["graph_ptr"] = np.asarray([0, num_nodes], dtype=np.int64)
    else:
        B = int(num_graphs if num_graphs is not None else (batch.max() + 1 if batch.size else 0))
        gp = np.zeros(B + 1, dtype=np.int64)
        gp[1:] = np.cumsum(np.bincount(batch, minlength=B)[:B])
        out["graph_ptr"] = gp
    return out


def _incidence(index: np.ndarray, n_rows: int, n_cols: int):
    """Sparse [n_rows, n_cols] matrix S with S[index[j], j] = 1 (scatter-sum operator)."""
    data = np.ones(index.shape[0], dtype=np.float64)
    return _sp.csr_matrix((data, (index, np.arange(index.shape[0]))), shape=(n_rows, n_cols))


def _scatter_sum(vals: np.ndarray, index: np.ndarray, n: int) -> np.ndarray:
    if _sp is not None:
        return np.asarray(_incidence(index, n, vals.shape[0]) @ vals)
    out = np.zeros((n,) + vals.shape[1:], dtype=vals.dtype)
    np.add.at(out, index, vals)
    return out


# ----------------------------------------------------------------------------------------------
# forward / backward
# ----------------------------------------------------------------------------------------------
def forward(params: dict, x, edge_index, edge_attr, batch, depth: int, act: str = "relu",
            learnable_skip: bool = False, num_graphs: int | None = None,
            dropout_masks: list | None = None, dropout_ps: list | None = None,
            relu_masks: dict | None = None, aggr: str = "add", pool: str = "add"):
    """GNN.forward (GNN.py:76-110) in float64. Returns (y[B], cache).

    ``aggr`` ("add" / "mean"): DMPNNConv's PyG aggregation (GNN.py:22,63,119); ``pool`` ("add" /
    "mean" / "max"): global_add_pool / global_mean_pool / global_max_pool (GNN.py:23,110).  PyG's
    mean is the sum divided by max(count, 1) (torch_geometric.utils.scatter, reduce="mean"), its
    max a column-wise amax: with a ``batch`` PyG runs ``scatter_reduce_(..., "amax",
    include_self=False)`` into zeros, whose backward shares a column's gradient evenly over the
    nodes holding the max and also counts the zero ``self`` when the max is 0 (torch
    FunctionsManual scatter_reduce_backward; checked against torch in tests/test_oracle_golden.py);
    with ``batch=None`` it is ``x.max(dim=-2)``, whose gradient goes to the first arg-max node.
    (PyG is absent here, its semantics restated.)

    ``params`` uses the reference ``state_dict`` keys.  ``dropout_masks[l]`` (optional, 0/1 per
    element of h) + ``dropout_ps[l]`` reproduce ``F.dropout`` in train mode with a given mask.
    ``relu_masks`` (ReLU only, optional): {"z0": [E,H], "zs": [D x [E,H]], "zn": [N,H]} boolean
    "z > 0" decisions to use instead of the fp64 signs -- the test-side reconciliation of
    pre-activations within rounding distance of 0, whose sign no fp32 implementation (the
    reference's own CPU path included) shares with fp64 (tests/test_gpu_parity.py).
    """
    f8 = np.float64
    x = np.asarray(x, dtype=f8)
    ea = np.asarray(edge_attr, dtype=f8)
    src = np.asarray(edge_index[0], dtype=np.int64)
    dst = np.asarray(edge_index[1], dtype=np.int64)
    N, E = x.shape[0], src.shape[0]
    assert E % 2 == 0, "reference view(E//2, 2, -1) needs an even edge count"
    W0 = np.asarray(params["edge_init.weight"], f8)
    b0 = np.asarray(params["edge_init.bias"], f8)
    sig = [float(np.asarray(params[f"skip_weights.{l}"])) if learnable_skip else 1.0
           for l in range(depth)]
    rev = np.arange(E) ^ 1
    assert aggr in ("add", "sum", "mean") and pool in ("add", "mean", "max")
    inv_deg = np.ones(N)
    if aggr == "mean":
        inv_deg = 1.0 / np.maximum(np.bincount(dst, minlength=N)[:N], 1)

    # GNN.py:85-87  h0 = act(edge_init(cat[x[row], edge_attr]))
    rm = relu_masks if (relu_masks is not None and act == "relu") else None

    def relu_or_mask(z, key, l=None):
        if rm is None:
            return act_fwd(z, act)
        mk = rm[key] if l is None else rm[key][l]
        return np.where(mk, z, 0.0)

    q0 = np.concatenate([x[src], ea], axis=1)
    z0 = q0 @ W0.T + b0
    h0 = relu_or_mask(z0, "z0")
    hs, As, zs, ms = [h0], [], [], []
    h = h0
    for l in range(depth):
        Wl = np.asarray(params[f"convs.{l}.lin.weight"], f8)
        bl = np.asarray(params[f"convs.{l}.lin.bias"], f8)
        a = _scatter_sum(h, dst, N) * inv_deg[:, None]  # GNN.py:134 propagate at edge_index[1]
        m = a[src] - h[rev]  # GNN.py:136-141
        z = m @ Wl.T + bl + sig[l] * h0  # GNN.py:141 + GNN.py:94-97
        hn = relu_or_mask(z, "zs", l)  # GNN.py:100-102
        if dropout_masks is not None and dropout_ps is not None and dropout_ps[l] > 0:
            hn = hn * dropout_masks[l] / (1.0 - dropout_ps[l])
        As.append(a)
        ms.append(m)
        zs.append(z)
        h = hn
        hs.append(h)
    s = _scatter_sum(h, dst, N) * inv_deg[:, None]  # GNN.py:105 (dead lin output dropped)
    Wn = np.asarray(params["edge_to_node.weight"], f8)
    bn = np.asarray(params["edge_to_node.bias"], f8)
    qn = np.concatenate([x, s], axis=1)  # GNN.py:106
    zn = qn @ Wn.T + bn
    hnode = relu_or_mask(zn, "zn")  # GNN.py:107
    if batch is None:
        g = hnode.sum(axis=0, keepdims=True)  # global_add_pool(h, None)
        gid = np.zeros(N, dtype=np.int64)
        B = 1
    else:
        gid = np.asarray(batch, dtype=np.int64)
        B = int(num_graphs if num_graphs is not None else gid.max() + 1)
        g = _scatter_sum(hnode, gid, B)  # GNN.py:110 global_add_pool
    inv_cnt = np.ones(B)
    pool_arg = None
    pool_share = None  # [N, H] each node's share of its column's gradient (max pool, batched)
    if pool == "mean":  # global_mean_pool
        inv_cnt = 1.0 / np.maximum(np.bincount(gid, minlength=B)[:B], 1)
        g = g * inv_cnt[:, None]
    elif pool == "max":  # global_max_pool: column max per graph
        g = np.zeros((B, hnode.shape[1]))
        pool_arg = np.full((B, hnode.shape[1]), -1, dtype=np.int64)
        for b in range(B):
            nodes = np.nonzero(gid == b)[0]
            if nodes.size:
                k = np.argmax(hnode[nodes], axis=0)  # first occurrence of the max
                pool_arg[b] = nodes[k]
                g[b] = hnode[nodes[k], np.arange(hnode.shape[1])]
        if batch is not None:  # scatter_reduce amax: ties share, the zero `self` counts at 0
            eq = hnode == g[gid]
            cnt = np.zeros((B, hnode.shape[1]))
            np.add.at(cnt, gid, eq.astype(np.float64))
            cnt = cnt + (g == 0.0)
            pool_share = np.where(eq, 1.0 / np.maximum(cnt[gid], 1.0), 0.0)
    wf = np.asarray(params["ffn.weight"], f8)  # [1, H]
    bf = np.asarray(params["ffn.bias"], f8)
    y = (g @ wf.T + bf)[:, 0]
    cache = dict(x=x, ea=ea, src=src, dst=dst, rev=rev, q0=q0, z0=z0, hs=hs, As=As, ms=ms,
                 zs=zs, s=s, qn=qn, zn=zn, hnode=hnode, g=g, gid=gid, B=B, sig=sig, N=N, E=E,
                 depth=depth, act=act, learnable_skip=learnable_skip,
                 masks=dropout_masks, ps=dropout_ps, relu_masks=rm, inv_deg=inv_deg,
                 inv_cnt=inv_cnt, pool_arg=pool_arg, pool_share=pool_share)
    return y, cache


def backward(params: dict, cache: dict, dy: np.ndarray, inputs_out: dict | None = None) -> dict:
    """Reverse mode of ``forward``. Returns grads keyed like ``state_dict``.
    ``inputs_out`` (a dict, optional) receives ``"x"`` [N, F] and ``"edge_attr"`` [E, Fe]."""
    f8 = np.float64
    act = cache["act"]
    D = cache["depth"]
    N, E = cache["N"], cache["E"]
    src, dst, rev = cache["src"], cache["dst"], cache["rev"]
    dy = np.asarray(dy, f8)
    grads = {}
    wf = np.asarray(params["ffn.weight"], f8)
    # head: y = g wf^T + bf
    grads["ffn.weight"] = (dy[None, :] @ cache["g"])  # [1, H]
    grads["ffn.bias"] = np.asarray([dy.sum()])
    dg = dy[:, None] * wf  # [B, H]
    rm = cache.get("relu_masks")

    def grad_of(z, key, l=None):
        if rm is None:
            return act_grad(z, act)
        mk = rm[key] if l is None else rm[key][l]
        return mk.astype(z.dtype)

    inv_deg, inv_cnt = cache["inv_deg"], cache["inv_cnt"]
    dhnode = (dg * inv_cnt[:, None])[cache["gid"]]  # pooling backward = gather by graph id
    if cache.get("pool_share") is not None:  # max pooling (batched): ties share the gradient
        dhnode = dhnode * cache["pool_share"]
    elif cache.get("pool_arg") is not None:  # max pooling, batch=None: the first arg-max node
        dhnode = dhnode * (cache["pool_arg"][cache["gid"]] == np.arange(N)[:, None])
    dzn = dhnode * grad_of(cache["zn"], "zn")
    grads["edge_to_node.weight"] = dzn.T @ cache["qn"]
    grads["edge_to_node.bias"] = dzn.sum(0)
    Wn = np.asarray(params["edge_to_node.weight"], f8)
    F_ = cache["x"].shape[1]
    ds = dzn @ Wn[:, F_:]  # [N, H]
    dh = (ds * inv_deg[:, None])[dst]  # readout aggregate backward: gather at dst
    dh0 = np.zeros_like(cache["hs"][0])
    for l in range(D - 1, -1, -1):
        z = cache["zs"][l]
        dz = dh * grad_of(z, "zs", l)
        if cache["masks"] is not None and cache["ps"] is not None and cache["ps"][l] > 0:
            dz = dh * cache["masks"][l] / (1.0 - cache["ps"][l]) * grad_of(z, "zs", l)
        Wl = np.asarray(params[f"convs.{l}.lin.weight"], f8)
        grads[f"convs.{l}.lin.weight"] = dz.T @ cache["ms"][l]
        grads[f"convs.{l}.lin.bias"] = dz.sum(0)
        if cache["learnable_skip"]:
            t = dz * cache["hs"][0]
            grads[f"skip_weights.{l}"] = np.asarray(t.sum())
            # sum |terms| of that scalar reduction: its conditioning (tests scale the bar by it)
            cache.setdefault("skip_abs", {})[f"skip_weights.{l}"] = float(np.abs(t).sum())
        dh0 += cache["sig"][l] * dz
        dm = dz @ Wl  # [E, H]
        da = _scatter_sum(dm, src, N)  # m = a[src] - h[rev]  ->  da = scatter_src(dm)
        dh = (da * inv_deg[:, None])[dst] - dm[rev]  # a = scatter_dst(h) ; rev: involution
    dh0 += dh
    dz0 = dh0 * grad_of(cache["z0"], "z0")
    grads["edge_init.weight"] = dz0.T @ cache["q0"]
    grads["edge_init.bias"] = dz0.sum(0)
    if inputs_out is not None:
        # q0 = [x[src] | e] (GNN.py:86): dq0 = dz0 W0; x[src] -> scatter at src; q = [x | s]
        dq0 = dz0 @ np.asarray(params["edge_init.weight"], f8)
        dx = _scatter_sum(dq0[:, :F_], src, N) + dzn @ Wn[:, :F_]
        inputs_out["x"] = dx
        inputs_out["edge_attr"] = dq0[:, F_:]
    return grads


def loss_and_grads(params, x, edge_index, edge_attr, batch, y_true, depth, act="relu",
                   learnable_skip=False, num_graphs=None, relu_masks=None, cache_out=None,
                   inputs_out=None, aggr="add", pool="add"):
    """MSELoss(reduction='sum') (train.py:120) forward + backward: (loss, y_hat, grads).
    `cache_out` (a dict, optional) receives the forward / backward cache (incl. "skip_abs");
    `inputs_out` (a dict, optional) the input gradients (``backward``)."""
    y, cache = forward(params, x, edge_index, edge_attr, batch, depth, act, learnable_skip,
                       num_graphs, relu_masks=relu_masks, aggr=aggr, pool=pool)
    r = y - np.asarray(y_true, np.float64)
    loss = float((r * r).sum())
    grads = backward(params, cache, 2.0 * r, inputs_out)
    if cache_out is not None:
        cache_out.update(cache)
    return loss, y, grads
